#!/bin/bash
# Round 3 final check of the committed tree: all GPU tests, smoke, the default bench line.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03t
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
cd "$R" || exit 1
step pytest 600 python3 -u -m pytest tests -m gpu -x -q --timeout 170 --timeout-method thread
step smoke 120 python3 -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python3 bench.py
