#!/bin/bash
# Placement bimodality, second counter set: UTCL1 translation, TCP->TCC latency, TA stalls.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r02pl2}
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
P="python3 $R/profiles/placement_pmc.py c4 6 1"
step p_tlb 200 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum TCP_UTCL1_STALL_MULTI_MISS_sum --output-format csv -d "$OUT/p_tlb" -o run -- $P
step p_lat 200 rocprofv3 --pmc TCP_TCC_WRITE_REQ_LATENCY_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_WRITE_REQ_sum TCP_TCC_READ_REQ_sum --output-format csv -d "$OUT/p_lat" -o run -- $P
step p_stall 200 rocprofv3 --pmc TCP_PENDING_STALL_CYCLES_sum TCP_UTCL1_THRASHING_STALL_sum TCP_UTCL1_SERIALIZATION_STALL_sum TCP_TCR_TCP_STALL_CYCLES_sum --output-format csv -d "$OUT/p_stall" -o run -- $P
step p_ta 200 rocprofv3 --pmc TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum --output-format csv -d "$OUT/p_ta" -o run -- $P
