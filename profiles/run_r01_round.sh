#!/bin/bash
# Round-1 GPU validation: all GPU tests, headline bench (+host-inclusive, +CPU baseline),
# and a 2-rank distributed rehearsal on one GPU (both ranks on device 0, reduced y extent).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r01b}
mkdir -p "$OUT"
cd "$R" || exit 1
timeout -k 10 600 python3 -m pytest tests -m gpu -q > "$OUT/gpu_tests.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/gpu_tests.log"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 500 python3 bench.py --host-inclusive > "$OUT/bench_c3.json" 2> "$OUT/bench_c3.err"
rc=$?; echo "bench rc=$rc"; cat "$OUT/bench_c3.json"; tail -3 "$OUT/bench_c3.err"
if [ $rc -ne 0 ]; then exit $rc; fi
ZH_DEVICE=0 timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 --ydiv 4 \
  > "$OUT/bench_2rank.json" 2> "$OUT/bench_2rank.err"
rc=$?; echo "2rank rc=$rc"; cat "$OUT/bench_2rank.json"; tail -3 "$OUT/bench_2rank.err"
exit $rc
