#!/bin/bash
# Round 3: GPU tests, then the aligned row-CRC tile decode with its end multiplies folded into
# one lane constant, against the unaligned kernel in one process (round-3 record: 35.44 vs
# 36.35 ms, profiles/r03/align/ab_align.json).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03i
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
cd /tmp || exit 1
step ab_c4crc_kq 500 python3 $R/profiles/ab_decode_env.py c4crc 1 5 - ZH_DEC_ALIGN=0
