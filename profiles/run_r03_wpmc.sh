#!/bin/bash
# Round 3: the write path's HBM traffic (c4 and c4crc encode): kernel trace + FETCH_SIZE and
# WRITE_SIZE passes of bench.py --op write, and the aligned decode's tests + A/B.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03w
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
cd /tmp || exit 1
B="python3 $R/bench.py --no-cpu-baseline --no-extras --no-host-inclusive --op write"
for cfg in c4crc c4; do
  step wtrace_$cfg 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/wtrace_$cfg" -o run -- $B --config $cfg --steps 3 --warmup 1
  step wfetch_$cfg 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/wfetch_$cfg" -o run -- $B --config $cfg --steps 2 --warmup 1
  step wwrite_$cfg 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/wwrite_$cfg" -o run -- $B --config $cfg --steps 2 --warmup 1
done
# c3crc: cached payload loads in the grouped row-CRC decode (ZH_CRC_LOADNT=0) vs non-temporal
B2="python3 $R/bench.py --no-cpu-baseline --no-extras --no-host-inclusive"
step ab_c3crc_nt 600 python3 $R/profiles/ab_decode_env.py c3crc 1 4 - ZH_CRC_LOADNT=0
step dtrace_c3crc 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_c3crc" -o run -- $B2 --config c3crc --steps 3 --warmup 1
step dfetch_c3crc 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch_c3crc" -o run -- $B2 --config c3crc --steps 2 --warmup 1
export ZH_CRC_LOADNT=0
step dfetch_c3crc_cached 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch_c3crccached" -o run -- $B2 --config c3crc --steps 2 --warmup 1
