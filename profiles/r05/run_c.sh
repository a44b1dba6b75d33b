#!/bin/bash
# Round 5 (c): the product multi-GPU pieces on one GPU (tests/test_gpu_parallel.py: read_device,
# RegionGather over a one-rank RCCL group), the file tests again after the O(1) descriptor
# eviction, and 2-rank rehearsals of the driver's strong and weak commands (ranks share the card:
# the gather rehearses through gloo, labelled).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${R05_TAG:-r05c}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  echo "== $name: $*" >&2
  timeout -k 10 "$t" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  echo "== $name rc=$rc" >&2
  if [ $rc -ne 0 ]; then tail -n 60 "$OUT/$name.out" "$OUT/$name.err" >&2; exit $rc; fi
}
cd "$R" || exit 1
step partests 300 python3 -u -m pytest tests/test_gpu_parallel.py tests/test_gpu_files.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider
step strong2 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --ydiv 4
step weak2 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --steps 5 --warmup 2 --ydiv 4 --mode weak
echo done >&2
