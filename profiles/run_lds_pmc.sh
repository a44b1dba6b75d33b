#!/bin/bash
# Kernel trace of the default bench (c4) with the current binary, plus LDS PMC passes
# (bank-conflict cycles vs all LDS-array cycles) on c4 and on the CRC-fused c4crc, whose
# tile kernel DESIGN §4 names LDS-bound.  Run on the GPU box from the repo root:
#   profiles/run_lds_pmc.sh [tag]
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r01lds}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
step() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  echo "== $name: $*" >&2
  timeout -k 10 "$t" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  echo "== $name rc=$rc" >&2
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step trace_c4 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_c4" -o run -- \
  python3 "$R/bench.py" --config c4 --steps 5 --warmup 2 --no-cpu-baseline --no-extras
for cfg in c4 c4crc; do
  step lds_$cfg 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES \
    --output-format csv -d "$OUT/lds_$cfg" -o run -- \
    python3 "$R/bench.py" --config $cfg --steps 1 --warmup 1 --no-cpu-baseline --no-extras
done
