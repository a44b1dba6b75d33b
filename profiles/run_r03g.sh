#!/bin/bash
# Round 3: GPU tests (compact-table tile CRC encode, 64 MiB default-kernel cases), the c3crc
# write path's kernel trace + FETCH/WRITE passes with cached stores, and a c4crc write A/B
# (compact tables at 4 workgroups per CU, tile groups of 1, the prefetching tile encode).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03g
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
cd /tmp || exit 1
step ab_c4crc_w 500 python3 $R/profiles/ab_write_env.py c4crc 1 3 - ZH_ENC_CRCLOW=1 ZH_ENC_CRCLOW=1,ZH_ENC_CRC_STNT=0 ZH_ENC_TPF=1
W="python3 $R/bench.py --no-cpu-baseline --no-extras --no-host-inclusive --op write"
cfg=c3crc
step wtrace_$cfg 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/wtrace_$cfg" -o run -- $W --config $cfg --steps 3 --warmup 1
step wfetch_$cfg 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/wfetch_$cfg" -o run -- $W --config $cfg --steps 2 --warmup 1
step wwrite_$cfg 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/wwrite_$cfg" -o run -- $W --config $cfg --steps 2 --warmup 1
step wsum_$cfg 60 python3 $R/profiles/pmc_summary_write.py "$OUT" $cfg "$OUT/write_${cfg}_summary.json" 206161575936
