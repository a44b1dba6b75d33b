#!/bin/bash
# Round 3: HIP API + kernel trace of the small one-shot read (profiles/small_read_trace.py).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03o
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
timeout -k 10 200 python3 $R/profiles/small_read_trace.py 200 > "$OUT/plain.out" 2> "$OUT/plain.err" && \
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 $R/profiles/small_read_trace.py 100 > "$OUT/trace.out" 2> "$OUT/trace.err"
