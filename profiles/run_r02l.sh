set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r02l
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "shuffled or concurren or gather" > $O/gpu_tests.log 2>&1 &&
timeout -k 10 500 python $R/bench.py --steps 20 --warmup 5 --cpu-budget 4 > $O/bench_n1.json 2> $O/bench_n1.err
