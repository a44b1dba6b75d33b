#!/bin/bash
# Round 6: the allocation-floor lab (profiles/r06/alloc_floor.py) on a third box, on the final
# tree, to check the default kind chosen from boxes 1 and 2.  Records → gpurun_out/r06alloc3.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r06alloc3
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R" || exit 1
timeout -k 5 60 amd-smi static -g 0 --json > "$OUT/amdsmi_static.json" 2>&1
timeout -k 10 480 python3 -u profiles/r06/alloc_floor.py "$OUT/alloc_floor.jsonl" 3 > "$OUT/alloc.out" 2> "$OUT/alloc.err"
rc=$?
echo "== alloc rc=$rc" >&2
tail -n 20 "$OUT/alloc.err" >&2
exit $rc
