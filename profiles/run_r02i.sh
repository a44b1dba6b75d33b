set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r02i
mkdir -p $O
timeout -k 10 500 python $R/bench.py --steps 20 --warmup 5 > $O/bench_n1.json 2> $O/bench_n1.err
