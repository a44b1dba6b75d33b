#!/bin/bash
# Round-1 final numbers on ONE box: GPU tests, the three configs, host-inclusive, CPU
# baseline, strong-scaling N=1, and 2-rank rehearsals (both ranks on device 0).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r01f}
mkdir -p "$OUT"
cd "$R" || exit 1
chk() { local rc=$1 name=$2; echo "$name rc=$rc"; if [ "$rc" -ne 0 ]; then tail -5 "$OUT/$name.err" 2>/dev/null; exit "$rc"; fi; }
timeout -k 10 600 python3 -m pytest tests -m gpu -q > "$OUT/gpu_tests.log" 2>&1; rc=$?
tail -2 "$OUT/gpu_tests.log"; chk $rc gpu_tests
timeout -k 10 500 python3 bench.py --config c3 --host-inclusive > "$OUT/bench_c3.json" 2> "$OUT/bench_c3.err"; chk $? bench_c3
timeout -k 10 300 python3 bench.py --config c4 --no-cpu-baseline > "$OUT/bench_c4.json" 2> "$OUT/bench_c4.err"; chk $? bench_c4
timeout -k 10 300 python3 bench.py --config c2 --no-cpu-baseline > "$OUT/bench_c2.json" 2> "$OUT/bench_c2.err"; chk $? bench_c2
timeout -k 10 300 python3 bench.py --mode strong --steps 5 > "$OUT/bench_strong1.json" 2> "$OUT/bench_strong1.err"; chk $? bench_strong1
ZH_DEVICE=0 timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29519 bench.py --gpus 2 --mode strong --ydiv 16 \
  --gather-backend gloo --steps 3 --warmup 1 > "$OUT/bench_strong2_gloo.json" 2> "$OUT/bench_strong2_gloo.err"
chk $? bench_strong2_gloo
ZH_DEVICE=0 timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29521 bench.py --gpus 2 --steps 3 --warmup 1 --ydiv 4 \
  > "$OUT/bench_weak2.json" 2> "$OUT/bench_weak2.err"
chk $? bench_weak2
for f in "$OUT"/bench_*.json; do echo "== $f"; cat "$f"; done
