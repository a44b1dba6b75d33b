#!/bin/bash
# Round 3: where the chunk-CRC tile encode spends its cycles — SQ counters (LDS instructions,
# bank-conflict cycles, LDS-array cycles, VALU instructions, busy cycles) for the c4 and
# c4crc write paths and the c4crc decode, one --pmc pass each (8 SQ + 1 GRBM counters).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03k
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
step() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  echo "== $name: $*" >&2
  timeout -s KILL "$t" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  echo "== $name rc=$rc" >&2
  if [ $rc -ne 0 ]; then exit $rc; fi
}
C="SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
B="python3 $R/bench.py --no-cpu-baseline --no-extras --no-host-inclusive --steps 1 --warmup 1"
step sq_w_c4crc 150 rocprofv3 --pmc $C --output-format csv -d "$OUT/sq_w_c4crc" -o run -- $B --op write --config c4crc
step sq_w_c4 150 rocprofv3 --pmc $C --output-format csv -d "$OUT/sq_w_c4" -o run -- $B --op write --config c4
step sq_r_c4crc 150 rocprofv3 --pmc $C --output-format csv -d "$OUT/sq_r_c4crc" -o run -- $B --config c4crc
