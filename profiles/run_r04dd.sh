#!/bin/bash
# Round 4, last tree: the default bench line, then the 2-rank weak-mode rehearsal at a quarter
# of the array (both ranks on the same card).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04dd
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  echo "== $name: $*" >&2
  timeout -k 10 "$t" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  echo "== $name rc=$rc" >&2
  if [ $rc -ne 0 ]; then tail -n 40 "$OUT/$name.out" "$OUT/$name.err" >&2; exit $rc; fi
}
cd "$R" || exit 1
step bench 400 python3 bench.py --steps 20 --warmup 5
step weak2 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --steps 5 --warmup 2 --ydiv 4 --mode weak
echo done >&2
