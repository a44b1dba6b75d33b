#!/bin/bash
# Round 3: 2-rank rehearsals of the driver's N>1 command on the one-GPU box (both ranks on
# device 0, reduced y extent): strong mode (the N>1 default: y-slabs, RCCL gather into the
# root's region, host-terminated slices) and weak mode (independent arrays per rank).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03h
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R" || exit 1
step() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  echo "== $name: $*" >&2
  timeout -k 10 "$t" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  echo "== $name rc=$rc" >&2
  tail -2 "$OUT/$name.err" >&2
  if [ $rc -ne 0 ]; then exit $rc; fi
}
export ZH_DEVICE=0
step strong2 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 3 --warmup 1 --ydiv 4
step weak2 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --ydiv 8 --mode weak
