#!/bin/bash
# Round 5: small one-plan reads into pageable memory staged through a page-locked buffer
# (ZH_HOUT_PIN, default 1): the GPU suite, the small-read A/B, the bench line.  Records → gpurun_out/r05hout.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05hout
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
step gputests 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step small_ab 300 python3 profiles/r05/small_ab.py "$OUT/small_hout_ab.json" 5 200 ZH_HOUT_PIN
cd /tmp || exit 1
step bench 400 python3 $R/bench.py
echo done >&2
