#!/bin/bash
# 2 MiB decode pieces as the default: the GPU suite, the c2 write A/B over the encode view's
# piece size, the default bench line (c4 headline + extras), and a c2 kernel trace.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${OUTD:-r02z}
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
step gpu_tests 600 python3 -u -m pytest $R/tests -m gpu -x -q --timeout 120 --timeout-method thread
step ab_write_c2 300 python3 -u $R/profiles/ab_write_env.py c2 1 3 - ZH_PIECE_KB=2048
step bench_n1 500 python3 $R/bench.py
cd /tmp || exit 1
step trace_c2 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_c2" -o run -- python3 $R/bench.py --no-cpu-baseline --no-extras --config c2 --steps 5 --warmup 2
