#!/bin/bash
# Placement bimodality, third counter set: where the writes go (DRAM vs GMI) and their stalls.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r02pl3}
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
step p_gmi 200 rocprofv3 --pmc TCC_EA0_WRREQ_WRITE_DRAM_32B_sum TCC_EA0_WRREQ_WRITE_GMI_32B_sum TCC_EA0_WRREQ_GMI_CREDIT_STALL_sum TCC_EA0_WRREQ_DRAM_sum --output-format csv -d "$OUT/p_gmi" -o run -- $P
step p_gmi2 200 rocprofv3 --pmc TCC_EA0_RDREQ_GMI_32B_sum TCC_EA0_RDREQ_DRAM_32B_sum TCC_EA0_RDREQ_GMI_CREDIT_STALL_sum TCC_EA0_WRREQ_IO_CREDIT_STALL_sum --output-format csv -d "$OUT/p_gmi2" -o run -- $P
