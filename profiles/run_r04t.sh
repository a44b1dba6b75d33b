#!/bin/bash
# Round 4: the file-source and concurrency tests, the write-files lab (mapped vs pwrite), then the GPU suite and smoke.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04t
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
step filetests 300 python3 -u -m pytest tests/test_gpu_concurrency.py tests/test_gpu_files.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider
step wlab 400 python3 -u profiles/write_files_lab.py $OUT/write_files_lab.json 3
step gputests 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step smoke 200 python3 -c "import __graft_entry__ as g; g.smoke()"
echo done >&2
