#!/bin/bash
# c2 (unsharded 1024^3 chunks, 4 KiB rows) knob sweep, interleaved in one process: piece size,
# 8 rows in flight per lane, item order; c3 item order with the lane exchange.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${OUTD:-r02y}
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
step ab_c2 400 python3 -u $R/profiles/ab_decode_env.py c2 1 5 - ZH_PIECE_KB=2048 ZH_PIECE_KB=4096 ZH_PIECE_KB=8192 ZH_PIECE_KB=2048,ZH_ITEM_PERM=1 ZH_PIECE_KB=4096,ZH_ITEM_PERM=1
step ab_c2le 300 python3 -u $R/profiles/ab_decode_env.py c2 1 3 - ZH_PIECE_KB=2048 ZH_PIECE_KB=8192,ZH_ITEM_PERM=1
