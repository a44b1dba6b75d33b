#!/bin/bash
# Round 5, seventh closing run: the last source tree (one plan for device-source host outputs
# below 1 GiB, the landing buffer bounded to 1 MiB): the GPU suite, the suite with one-launch
# small plans forced on, smoke, the default bench line, the c4 kernel trace.
# Records → gpurun_out/r05final7.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05final7
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
step gputests 800 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
export ZH_SMALL_ONE=1
step gputests_small_one 800 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
unset ZH_SMALL_ONE
step smoke 200 python3 -c "import __graft_entry__ as g; g.smoke()"
step bench 500 python3 bench.py --steps 20 --warmup 5
cd /tmp || exit 1
B="python3 $R/bench.py --no-cpu-baseline --no-extras --no-host-inclusive"
step trace_c4 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_c4" -o run -- $B --config c4 --steps 5 --warmup 2
echo done >&2
