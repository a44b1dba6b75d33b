#!/bin/bash
# Round 5: device-source reads into host memory take one plan below ZH_PIPE_DOUT_MIN_KB (1 GiB):
# the GPU suite, then the pipelined-vs-one-plan A/B at 64-512 MiB and 1-2 GiB.
# Records → gpurun_out/mid.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/mid
mkdir -p "$OUT"
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
export MID_VAR=ZH_PIPE_DOUT_MIN_KB
export MID_BIG=1
step big_ab2 300 python3 profiles/r05/mid_ab.py "$OUT/big_ab2.json" 3 10
unset MID_BIG
export MID_HUGE=1
step huge_ab 300 python3 profiles/r05/mid_ab.py "$OUT/huge_ab.json" 3 5
echo done >&2
