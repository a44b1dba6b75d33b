#!/bin/bash
# Round 4: the JNI shim executed under the fake JVM on the GPU (tests/test_jni_shim.py, the whole
# GPU suite after the host index check / piece-overlap changes), then the critical-window lab
# (profiles/jni_window_lab.py: the 2 GiB sub-shard read through arrayReadPieces per slab cap).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04b
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
step jnitests 300 python3 -u -m pytest tests/test_jni_shim.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider
step gputests 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step jnilab 400 python3 -u profiles/jni_window_lab.py "$OUT/jni_window_lab.json"
echo done >&2
