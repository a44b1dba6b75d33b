#!/bin/bash
# Round 3 closing run: all GPU tests and smoke; the aligned row-CRC decode over field tables
# (ZH_DEC_CRCFIELD=1) A/B and its SQ pass; the headline c4 kernel trace + FETCH/WRITE passes
# with the closing binary (summary made on the box); the default bench line.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03n
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
step smoke 120 python3 -c "import __graft_entry__ as g; g.smoke()"
cd /tmp || exit 1
step ab_c4crc_dfield 500 python3 $R/profiles/ab_decode_env.py c4crc 1 5 - ZH_DEC_CRCFIELD=1
C="SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
P="python3 $R/bench.py --no-cpu-baseline --no-extras --no-host-inclusive"
export ZH_DEC_CRCFIELD=1
step sq_r_c4crc_field 150 rocprofv3 --pmc $C --output-format csv -d "$OUT/sq_r_c4crc_field" -o run -- $P --steps 1 --warmup 1 --config c4crc
unset ZH_DEC_CRCFIELD
cfg=c4
step trace_$cfg 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_$cfg" -o run -- $P --config $cfg --steps 5 --warmup 2
step pmc_fetch_$cfg 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch_$cfg" -o run -- $P --config $cfg --steps 2 --warmup 1
step pmc_write_$cfg 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write_$cfg" -o run -- $P --config $cfg --steps 2 --warmup 1
step sum_$cfg 60 python3 $R/profiles/pmc_summary.py "$OUT" $cfg "$OUT/${cfg}_summary.json"
cd "$R" || exit 1
step bench 600 python3 bench.py
