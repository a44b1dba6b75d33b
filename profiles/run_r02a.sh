set -o pipefail
mkdir -p gpurun_out/r02a
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02a/gpu_tests.log 2>&1 &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02a/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r02a/bench_c4.json 2> gpurun_out/r02a/bench_c4.err
