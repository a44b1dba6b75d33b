#!/bin/bash
# Round-2 profiles with the final binary: kernel trace + stats per config, FETCH_SIZE and
# WRITE_SIZE in separate --pmc passes (c4, c3, c2), the CRC configs' traces, write benches.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r02p
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
B="python3 $R/bench.py --no-cpu-baseline --no-extras"
for cfg in c4 c3 c2; do
  step trace_$cfg 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_$cfg" -o run -- $B --config $cfg --steps 5 --warmup 2
  step pmc_fetch_$cfg 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch_$cfg" -o run -- $B --config $cfg --steps 2 --warmup 1
  step pmc_write_$cfg 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write_$cfg" -o run -- $B --config $cfg --steps 2 --warmup 1
done
for cfg in c4crc c3crc c3nest; do
  step trace_$cfg 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_$cfg" -o run -- $B --config $cfg --steps 5 --warmup 2
done
for cfg in c4 c3 c2 c4crc c3crc; do
  step write_$cfg 300 $B --config $cfg --op write --steps 5 --warmup 2
done
