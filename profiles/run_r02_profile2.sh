#!/bin/bash
# Round-2 profiles after the lane-exchange row decode and the arena pair: kernel trace + stats
# (c4, c3, c3nest), FETCH_SIZE and WRITE_SIZE in separate --pmc passes (c4, c3).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r02p2
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
for cfg in c4 c3; do
  step trace_$cfg 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_$cfg" -o run -- $B --config $cfg --steps 5 --warmup 2
  step pmc_fetch_$cfg 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch_$cfg" -o run -- $B --config $cfg --steps 2 --warmup 1
  step pmc_write_$cfg 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write_$cfg" -o run -- $B --config $cfg --steps 2 --warmup 1
done
step trace_c3nest 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_c3nest" -o run -- $B --config c3nest --steps 5 --warmup 2
