set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r02g
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 &&
timeout -k 10 300 python $R/bench.py --gpus 2 --ydiv 4 --steps 10 --warmup 2 > $O/bench_n2_rehearsal.json 2> $O/bench_n2_rehearsal.err
