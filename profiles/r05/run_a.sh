#!/bin/bash
# Round 5 (a): the store-path changes (zero-padded part reads, readFailed text, bounded
# descriptors, atomic chunk writes, typed file sources) on the GPU: the file / JNI / pieces
# tests first, then the whole GPU suite, smoke, and the default bench line.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05a
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
step filetests 400 python3 -u -m pytest tests/test_gpu_files.py tests/test_jni_shim.py tests/test_gpu_pieces.py tests/test_gpu_concurrency.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider
step gputests 700 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step smoke 200 python3 -c "import __graft_entry__ as g; g.smoke()"
step bench 500 python3 bench.py --steps 20 --warmup 5
echo done >&2
