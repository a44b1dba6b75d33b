#!/bin/bash
# Placement bimodality: L2-channel and XCC distribution of the decode's memory-side writes.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r02pl4}
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
CH=$(seq -s ' ' -f 'ZH_WRCH%g' 0 15)
XC=$(seq -s ' ' -f 'ZH_WRXCC%g' 0 7)
step p_ch 200 rocprofv3 -E "$R/profiles/pmc_channels.yaml" --pmc $CH --output-format csv -d "$OUT/p_ch" -o run -- $P
step p_xcc 200 rocprofv3 -E "$R/profiles/pmc_channels.yaml" --pmc $XC --output-format csv -d "$OUT/p_xcc" -o run -- $P
