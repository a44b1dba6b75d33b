#!/bin/bash
# Row-CRC tile kernel on the encode view (ZH_ENC_ROWCRC=1): CRC/encode parity tests, then an
# interleaved full-size c4crc write A/B against the fused grouped tile encode.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${OUTD:-r02x}
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
step tests 300 python3 -u -m pytest $R/tests/test_gpu_parity.py $R/tests/test_gpu_crc_tiles.py -m gpu -x -q --timeout 120 --timeout-method thread
step ab_write 400 python3 -u $R/profiles/ab_write_env.py c4crc 1 5 - ZH_ENC_ROWCRC=1 ZH_ENC_ROWCRC=1,ZH_ENC_TGROUP=1 ZH_ENC_ROWCRC=1,ZH_ENC_TGROUP=4
