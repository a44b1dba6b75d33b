#!/bin/bash
# Round-2 closing profiles with the final binary: kernel trace + stats and FETCH_SIZE /
# WRITE_SIZE passes (separate runs) for c4 (the metric) and c2 (2 MiB work items).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r02final
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
step() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  echo "== $name: $*" >&2
  timeout -k 10 "$t" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  echo "== $name rc=$rc" >&2
  if [ $rc -ne 0 ]; then exit $rc; fi
}
B="python3 $R/bench.py --no-cpu-baseline --no-extras"
for cfg in c4 c2; do
  step trace_$cfg 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_$cfg" -o run -- $B --config $cfg --steps 5 --warmup 2
  step pmc_fetch_$cfg 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch_$cfg" -o run -- $B --config $cfg --steps 2 --warmup 1
  step pmc_write_$cfg 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write_$cfg" -o run -- $B --config $cfg --steps 2 --warmup 1
done
