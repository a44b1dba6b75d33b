#!/bin/bash
# Round 3: the grouped row-CRC decode with 8 rows per lane in flight (ZH_DEC_RGU=8): parity
# tests, then an interleaved c3crc decode A/B.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03u
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
step pytest 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 170 --timeout-method thread -k "row_crc or crc"
cd /tmp || exit 1
step ab_c3crc_rgu 500 python3 $R/profiles/ab_decode_env.py c3crc 1 5 - ZH_DEC_RGU=8
