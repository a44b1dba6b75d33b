#!/bin/bash
# Round 4: HIP API + kernel trace of the 64^3 store read (zh_array_read_files, one plan).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04s
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 "$R/profiles/small_store_lab.py" "$OUT/lab.json" 100 trace > "$OUT/trace.out" 2> "$OUT/trace.err" || { tail -20 "$OUT/trace.err" >&2; exit 1; }
echo done >&2
