#!/bin/bash
# Kernel trace + stats of the write path (c3, c4): which kernels the 40 ms encode spends in.
#   profiles/run_write_trace.sh [tag]   (GPU box, repo root)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r02wt}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
for cfg in ${CONFIGS:-c3 c4}; do
  echo "== write $cfg" >&2
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/wtrace_$cfg" -o run -- \
    python3 "$R/bench.py" --op write --config $cfg --steps 5 --warmup 2 --no-cpu-baseline --no-extras \
    > "$OUT/wtrace_$cfg.out" 2> "$OUT/wtrace_$cfg.err" || exit $?
done
