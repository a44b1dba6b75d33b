#!/bin/bash
# Round-3 closing profiles with the current binary: kernel trace + stats and FETCH_SIZE /
# WRITE_SIZE passes (separate runs) for the decode of c4 (the metric), c4crc and c3crc, and for
# the write path (bench.py --op write) of c4crc and c3crc; write-path traces of c4 and c3; then
# the CRC encodes' cached-store A/B (ZH_ENC_CRC_STNT=0).  Summaries are made on the box.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03final
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
B="python3 $R/bench.py --no-cpu-baseline --no-extras --no-host-inclusive"
for cfg in c4 c4crc c3crc; do
  step trace_$cfg 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_$cfg" -o run -- $B --config $cfg --steps 5 --warmup 2
  step pmc_fetch_$cfg 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch_$cfg" -o run -- $B --config $cfg --steps 2 --warmup 1
  step pmc_write_$cfg 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write_$cfg" -o run -- $B --config $cfg --steps 2 --warmup 1
  step sum_$cfg 60 python3 $R/profiles/pmc_summary.py "$OUT" $cfg "$OUT/${cfg}_summary.json"
done
W="$B --op write"
for cfg in c4crc c3crc; do
  step wtrace_$cfg 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/wtrace_$cfg" -o run -- $W --config $cfg --steps 3 --warmup 1
  step wfetch_$cfg 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/wfetch_$cfg" -o run -- $W --config $cfg --steps 2 --warmup 1
  step wwrite_$cfg 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/wwrite_$cfg" -o run -- $W --config $cfg --steps 2 --warmup 1
  step wsum_$cfg 60 python3 $R/profiles/pmc_summary_write.py "$OUT" $cfg "$OUT/write_${cfg}_summary.json" 206161575936
done
for cfg in c4 c3; do
  step wtrace_$cfg 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/wtrace_$cfg" -o run -- $W --config $cfg --steps 3 --warmup 1
done
step ab_stnt_c3crc 400 python3 $R/profiles/ab_write_env.py c3crc 1 3 - ZH_ENC_CRC_STNT=0
step ab_stnt_c4crc 400 python3 $R/profiles/ab_write_env.py c4crc 1 3 - ZH_ENC_CRC_STNT=0
