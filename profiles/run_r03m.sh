#!/bin/bash
# Round 3: the aligned row-CRC tile decode over conflict-free field tables (ZH_DEC_CRCFIELD=1):
# CRC tile tests, an interleaved c4crc decode A/B and an SQ counter pass of it.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03m
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
step pytest 300 python3 -u -m pytest tests/test_gpu_crc_tiles.py -x -q --timeout 170 --timeout-method thread
cd /tmp || exit 1
step ab_c4crc_dfield 500 python3 $R/profiles/ab_decode_env.py c4crc 1 5 - ZH_DEC_CRCFIELD=1
C="SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
export ZH_DEC_CRCFIELD=1
step sq_r_c4crc_field 150 rocprofv3 --pmc $C --output-format csv -d "$OUT/sq_r_c4crc_field" -o run -- python3 $R/bench.py --no-cpu-baseline --no-extras --no-host-inclusive --steps 1 --warmup 1 --config c4crc
