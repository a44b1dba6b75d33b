#!/bin/bash
# Row-CRC tile kernel as the c4crc default: the whole GPU suite, the c4crc bench line and its
# rocprofv3 kernel trace + stats, plus FETCH_SIZE / WRITE_SIZE passes (traffic per launch).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r02v
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  echo "== $name: $*" >&2
  timeout -k 10 "$t" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  echo "== $name rc=$rc" >&2
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step gpu_tests 600 python3 -u -m pytest $R/tests -m gpu -x -q --timeout 120 --timeout-method thread
cd /tmp || exit 1
B="python3 $R/bench.py --no-cpu-baseline --no-extras"
step bench_c4crc 300 $B --config c4crc
step trace_c4crc 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_c4crc" -o run -- $B --config c4crc --steps 5 --warmup 2
step pmc_fetch_c4crc 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch_c4crc" -o run -- $B --config c4crc --steps 2 --warmup 1
step pmc_write_c4crc 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write_c4crc" -o run -- $B --config c4crc --steps 2 --warmup 1
