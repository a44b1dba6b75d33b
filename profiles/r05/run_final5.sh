#!/bin/bash
# Round 5, fifth closing run (after the fused index CRC and the one-launch small plans):
# the GPU suite, smoke, the default bench line, kernel traces and PMC passes of the c4 / c3 / c2
# decodes and the c4crc / c3crc encodes.  Records → gpurun_out/r05final5.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05final5
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  echo "== $name: $*" >&2
  timeout -k 10 "$t" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  echo "== $name rc=$rc" >&2
  if [ $rc -ne 0 ]; then tail -n 60 "$OUT/$name.out" "$OUT/$name.err" >&2; exit $rc; fi
}
cd "$R" || exit 1
step gputests 800 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step smoke 200 python3 -c "import __graft_entry__ as g; g.smoke()"
step bench 500 python3 bench.py --steps 20 --warmup 5
cd /tmp || exit 1
B="python3 $R/bench.py --no-cpu-baseline --no-extras --no-host-inclusive"
step trace_c4 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_c4" -o run -- $B --config c4 --steps 5 --warmup 2
step pmc_fetch_c4 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch_c4" -o run -- $B --config c4 --steps 2 --warmup 1
step pmc_write_c4 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write_c4" -o run -- $B --config c4 --steps 2 --warmup 1
step sum_c4 60 python3 $R/profiles/pmc_summary.py "$OUT" c4 "$OUT/c4_summary.json"
for cfg in c3 c2; do
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
echo done >&2
