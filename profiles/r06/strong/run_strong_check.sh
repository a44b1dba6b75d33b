#!/bin/bash
# Round 6: bench.py's N > 1 strong-mode code path after its change (each rank's copy ceiling),
# two ranks on this one GPU at a quarter of the array (--ydiv 4; the full-size gloo gather needs
# more host memory than one box has, and now says so instead).  A code-path check, not scaling
# evidence.  Records → gpurun_out/r06strong.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r06strong
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R" || exit 1
timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --ydiv 4 --no-host-out > "$OUT/strong2.out" 2> "$OUT/strong2.err"
rc=$?
echo "== strong2 rc=$rc" >&2
tail -n 30 "$OUT/strong2.err" >&2
exit $rc
