#!/bin/bash
# Round 4: zh_array_read_files knobs (in/out lanes, ring window, slab size) on the sub-shard and
# two-shard store reads (profiles/files_lab.py).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04k
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  echo "== $name: $*" >&2
  timeout -k 10 "$t" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  echo "== $name rc=$rc" >&2
  if [ $rc -ne 0 ]; then tail -n 40 "$OUT/$name.out" "$OUT/$name.err" >&2; exit $rc; fi
}
cd "$R" || exit 1
step fileslab 500 python3 -u profiles/files_lab.py "$OUT/files_lab.json" 5
echo done >&2
