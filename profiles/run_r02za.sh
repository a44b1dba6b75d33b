#!/bin/bash
# 2 MiB pieces on the encode view too: the GPU suite and the c2 / c3 write bench lines.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${OUTD:-r02za}
mkdir -p "$OUT"
step() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  echo "== $name: $*" >&2
  timeout -k 10 "$t" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  echo "== $name rc=$rc" >&2
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step gpu_tests 600 python3 -u -m pytest $R/tests -m gpu -x -q --timeout 120 --timeout-method thread
step write_c2 300 python3 $R/bench.py --no-cpu-baseline --no-extras --config c2 --op write --steps 5 --warmup 2
step write_c3 300 python3 $R/bench.py --no-cpu-baseline --no-extras --config c3 --op write --steps 5 --warmup 2
