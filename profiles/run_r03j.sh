#!/bin/bash
# Round 3: GPU tests and smoke, the default bench line (now with small_read), the c4crc and
# c3crc decode and write lines with the current binary; c4crc decode profiles (trace + PMC)
# and its write-path trace.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03j
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
step smoke 120 python3 -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python3 bench.py
B="python3 bench.py --no-cpu-baseline --no-extras --no-host-inclusive"
step c4crc_read 300 $B --config c4crc
step c3crc_read 300 $B --config c3crc
step c4crc_write 300 $B --config c4crc --op write --steps 5 --warmup 2
step c3crc_write 300 $B --config c3crc --op write --steps 5 --warmup 2
cd /tmp || exit 1
step ab_c3crc_group 500 python3 $R/profiles/ab_write_env.py c3crc 1 3 - ZH_ENC_GROUP=4 ZH_ENC_GROUP=1
P="python3 $R/bench.py --no-cpu-baseline --no-extras --no-host-inclusive"
cfg=c4crc
step trace_$cfg 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_$cfg" -o run -- $P --config $cfg --steps 5 --warmup 2
step pmc_fetch_$cfg 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch_$cfg" -o run -- $P --config $cfg --steps 2 --warmup 1
step pmc_write_$cfg 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write_$cfg" -o run -- $P --config $cfg --steps 2 --warmup 1
step sum_$cfg 60 python3 $R/profiles/pmc_summary.py "$OUT" $cfg "$OUT/${cfg}_summary.json"
step wtrace_$cfg 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/wtrace_$cfg" -o run -- $P --op write --config $cfg --steps 3 --warmup 1
