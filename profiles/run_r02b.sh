set -o pipefail
mkdir -p gpurun_out/r02b
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/r02b/bench_n1.json 2> gpurun_out/r02b/bench_n1.err &&
timeout -k 10 300 python bench.py --gpus 2 --ydiv 4 --steps 10 --warmup 2 > gpurun_out/r02b/bench_n2_rehearsal.json 2> gpurun_out/r02b/bench_n2_rehearsal.err
