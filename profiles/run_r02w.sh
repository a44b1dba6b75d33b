#!/bin/bash
# SDWA table lookups (tables at a constant LDS position) in the CRC row and tile group kernels:
# the GPU suite, then c3crc decode + the two CRC writes and the fused c4crc (ZH_DEC_CRCW=0).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${OUTD:-r02w}
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
step gpu_tests 600 python3 -u -m pytest $R/tests -m gpu -x -q --timeout 120 --timeout-method thread
B="python3 $R/bench.py --no-cpu-baseline --no-extras"
step bench_c3crc 300 $B --config c3crc
step write_c3crc 300 $B --config c3crc --op write --steps 5 --warmup 2
step write_c4crc 300 $B --config c4crc --op write --steps 5 --warmup 2
step ab_c4crc 300 python3 -u $R/profiles/ab_decode_env.py c4crc 1 5 - ZH_DEC_CRCW=0
