#!/bin/bash
# Round 3: GPU tests (incl. the index-CRC split combine), then the small one-shot read with the
# index CRC combined by the last workgroup (default) or by a second launch (ZH_CRC_SPLIT=1).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03q
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
cd "$R" || exit 1
step pytest 600 python3 -u -m pytest tests -m gpu -x -q --timeout 170 --timeout-method thread
step ab_small 300 python3 profiles/small_read_ab.py 200 - ZH_CRC_SPLIT=1
step ab_c4 500 python3 profiles/ab_decode_env.py c4 1 3 - ZH_CRC_SPLIT=1
