#!/bin/bash
# Round 6: the GPU suite, smoke and the c4crc / c4 write and c4 read lines with the deferred
# CRC fold in the tile encode (the plain encode's loads now sit in their own live branch).
# Records → gpurun_out/r06verify2.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r06verify2
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
B="python3 bench.py --no-cpu-baseline --no-extras --no-host-inclusive --allocations 1"
step write_c4crc 300 $B --op write --config c4crc --steps 5 --warmup 2
step write_c4 300 $B --op write --config c4 --steps 5 --warmup 2
step read_c4 300 $B --config c4 --steps 10 --warmup 3
echo done >&2
