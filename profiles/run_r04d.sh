#!/bin/bash
# Round 4: the GPU suite with the pipeline's minimum slab count, the JNI critical-window lab again
# (mid-sized pipelined reads now run in >= 8 slabs), the default bench line, and the 2-rank
# strong-mode rehearsal at a quarter of the array (--ydiv 4: ranks share the card, so gloo
# through host memory stands in for RCCL; the full size exceeds the box's host-memory cap).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04d
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
step gputests 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step jnilab 400 python3 -u profiles/jni_window_lab.py "$OUT/jni_window_lab.json"
step bench 400 python3 bench.py --steps 20 --warmup 5
step strong2 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --ydiv 4
echo done >&2
