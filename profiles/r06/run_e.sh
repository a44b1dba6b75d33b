#!/bin/bash
# Round 6: the sector-aligned chunk-CRC tile encode — its tests first (small sizes, stop at the
# first failure), then the c4crc write under the kernel trace and the PMC write/fetch passes.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${RUN_TAG:-r06e}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  echo "== $name: $*" >&2
  timeout -k 10 "$t" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  echo "== $name rc=$rc" >&2
  if [ $rc -ne 0 ]; then tail -n 60 "$OUT/$name.out" "$OUT/$name.err" >&2; exit $rc; fi
}
cd "$R" || exit 1
step tests 600 python3 -u -m pytest tests/test_gpu_crc_tiles.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
cd /tmp || exit 1
W="python3 $R/bench.py --no-cpu-baseline --no-extras --no-host-inclusive --op write --config c4crc"
step wbench 300 $W --steps 5 --warmup 2
step wtrace 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/wtrace_c4crc" -o run -- $W --steps 3 --warmup 1
step wfetch 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/wfetch_c4crc" -o run -- $W --steps 2 --warmup 1
step wwrite 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/wwrite_c4crc" -o run -- $W --steps 2 --warmup 1
step wsum 60 python3 $R/profiles/pmc_summary_write.py "$OUT" c4crc "$OUT/write_c4crc_summary.json" 206161575936
echo done >&2
