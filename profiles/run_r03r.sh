#!/bin/bash
# Round 3: small one-shot read vs the index-CRC span per workgroup (ZH_CRC_SHIFT: 4 KiB << s),
# and the CRC tile tests under the largest span.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03r
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
step ab_small_shift 300 python3 profiles/small_read_ab.py 200 - ZH_CRC_SHIFT=1 ZH_CRC_SHIFT=2 ZH_CRC_SHIFT=3 ZH_CRC_SHIFT=4
ZH_CRC_SHIFT=2 step pytest_shift2 300 env ZH_CRC_SHIFT=2 python3 -u -m pytest tests/test_gpu_crc_tiles.py tests/test_gpu_parity.py -x -q --timeout 170 --timeout-method thread
