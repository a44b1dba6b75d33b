#!/bin/bash
# Placement bimodality, counters per dispatch: timing run, then one rocprofv3
# --pmc pass per counter group over the same script.  usage: profiles/run_placement_pmc.sh [tag]
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r02pl}
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
step time 200 python3 "$R/profiles/placement_pmc.py" c4 6 3
step pmc_req 200 rocprofv3 --pmc TCC_EA0_WRREQ TCC_EA0_RDREQ --output-format csv -d "$OUT/pmc_req" -o run -- \
  python3 "$R/profiles/placement_pmc.py" c4 6 1
step pmc_wstall 200 rocprofv3 --pmc TCC_EA0_WRREQ_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_TOO_MANY_EA_WRREQS_STALL_sum TCC_TAG_STALL_sum --output-format csv -d "$OUT/pmc_wstall" -o run -- \
  python3 "$R/profiles/placement_pmc.py" c4 6 1
step pmc_rstall 200 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_LEVEL_sum TCC_EA0_RDREQ_LEVEL_sum TCC_BUBBLE_sum --output-format csv -d "$OUT/pmc_rstall" -o run -- \
  python3 "$R/profiles/placement_pmc.py" c4 6 1
