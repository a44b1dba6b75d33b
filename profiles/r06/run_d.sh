#!/bin/bash
# Round 6: the allocation tests with the new default kind, the default bench line (1 GiB
# chunks for the output and the slab), then the chunk-CRC encode cache-policy lab.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r06d
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
step alloc_tests 300 python3 -u -m pytest tests/test_gpu_alloc.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step bench 500 python3 bench.py --steps 10 --warmup 3
bash "$R/profiles/r06/run_enc.sh" || exit $?
echo done >&2
