#!/bin/bash
# Round 6: the file tests after the ADVICE fixes, then the allocation-floor lab on this box.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r06c
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  echo "== $name: $*" >&2
  timeout -k 10 "$t" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  echo "== $name rc=$rc" >&2
  if [ $rc -ne 0 ]; then tail -n 60 "$OUT/$name.out" "$OUT/$name.err" >&2; exit $rc; fi
}
cd "$R" || exit 1
timeout -k 5 60 amd-smi static -g 0 --json > "$OUT/amdsmi_static.json" 2>&1
step files 400 python3 -u -m pytest tests/test_gpu_files.py tests/test_gpu_multi.py tests/test_gpu_parallel.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step alloc 420 python3 -u profiles/r06/alloc_floor.py "$OUT/alloc_floor.jsonl" 3
echo done >&2
