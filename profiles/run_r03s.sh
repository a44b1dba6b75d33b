#!/bin/bash
# Round 3: where the waves of the tile kernels spend their cycles (WAIT_ANY + WAIT_INST_ANY +
# ACTIVE_INST_ANY = WAVE_CYCLES; the guide's SQ table): c4 / c4crc, write and read.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03s
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
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
B="python3 $R/bench.py --no-cpu-baseline --no-extras --no-host-inclusive --steps 1 --warmup 1"
step w_c4crc 150 rocprofv3 --pmc $C --output-format csv -d "$OUT/w_c4crc" -o run -- $B --op write --config c4crc
step w_c4 150 rocprofv3 --pmc $C --output-format csv -d "$OUT/w_c4" -o run -- $B --op write --config c4
step r_c4crc 150 rocprofv3 --pmc $C --output-format csv -d "$OUT/r_c4crc" -o run -- $B --config c4crc
step r_c3crc 150 rocprofv3 --pmc $C --output-format csv -d "$OUT/r_c3crc" -o run -- $B --op write --config c3crc
