#!/bin/bash
# Round 5: the chunk-crc32c decode configs with this round's binary:
# bench lines and kernel traces for c4crc / c3crc.  Records → gpurun_out/r05crc.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05crc
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
cd /tmp || exit 1
B="python3 $R/bench.py --no-cpu-baseline --no-extras --no-host-inclusive"
for cfg in c4crc c3crc; do
  step bench_$cfg 300 $B --config $cfg --steps 20 --warmup 5
  step trace_$cfg 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_$cfg" -o run -- $B --config $cfg --steps 5 --warmup 2
done
echo done >&2
