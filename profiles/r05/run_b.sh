#!/bin/bash
# Round 5 (b): allocation A/B of the decode (hipMalloc vs 1 GiB VMM chunks, output and shard
# slab separately) for c4 and c2 in one process each, then the default bench line again.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05b
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  echo "== $name: $*" >&2
  timeout -k 10 "$t" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  echo "== $name rc=$rc" >&2
  if [ $rc -ne 0 ]; then tail -n 40 "$OUT/$name.out" "$OUT/$name.err" >&2; exit $rc; fi
}
cd "$R" || exit 1
step ab_c4 300 python3 -u profiles/r05/alloc_ab.py c4 "$OUT/alloc_ab_c4.json"
step ab_c2 300 python3 -u profiles/r05/alloc_ab.py c2 "$OUT/alloc_ab_c2.json"
step bench 500 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline
echo done >&2
