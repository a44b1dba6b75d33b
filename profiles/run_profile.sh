#!/bin/bash
# Profiling recipe (run on the GPU box from the repo root):
#   per config: kernel trace + stats of the bench, then separate PMC passes for HBM bytes
#   (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950).
#   usage: profiles/run_profile.sh [tag] ; CONFIGS="c3 c4 c2" by default
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r01}
OUT=$R/gpurun_out/$TAG
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
for cfg in ${CONFIGS:-c3 c4 c2}; do
  step trace_$cfg 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_$cfg" -o run -- \
    python3 "$R/bench.py" --config $cfg --steps 5 --warmup 2 --no-cpu-baseline --no-extras
  step pmc_fetch_$cfg 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch_$cfg" -o run -- \
    python3 "$R/bench.py" --config $cfg --steps 2 --warmup 1 --no-cpu-baseline --no-extras
  step pmc_write_$cfg 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write_$cfg" -o run -- \
    python3 "$R/bench.py" --config $cfg --steps 2 --warmup 1 --no-cpu-baseline --no-extras
done
