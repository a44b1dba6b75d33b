#!/bin/bash
# Round 3: CRC tile tests with the lane-constant fold in the row-CRC tile kernel, then the
# row-CRC tile encode (ZH_ENC_ROWCRC=1; 2, 4 and 1 chunks per work item) against the default
# fused tile encode, c4crc write, one process.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03v
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
step pytest 400 python3 -u -m pytest tests/test_gpu_crc_tiles.py tests/test_gpu_parity.py -x -q --timeout 170 --timeout-method thread
cd /tmp || exit 1
step ab 600 python3 $R/profiles/ab_write_env.py c4crc 1 3 - ZH_ENC_ROWCRC=1 ZH_ENC_ROWCRC=1,ZH_ENC_TGROUP=4 ZH_ENC_ROWCRC=1,ZH_ENC_TGROUP=1
