set -o pipefail
mkdir -p gpurun_out/r02e
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/r02e/bench_scatter.json 2> gpurun_out/r02e/bench_scatter.err &&
ZH_MALLOC=0 timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r02e/bench_plain.json 2> gpurun_out/r02e/bench_plain.err
