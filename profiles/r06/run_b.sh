set -o pipefail
mkdir -p gpurun_out/r06b
(timeout -k 5 60 amd-smi metric -g 0 --json > gpurun_out/r06b/amdsmi_metric.json 2> gpurun_out/r06b/amdsmi_metric.err; timeout -k 5 60 amd-smi static -g 0 --json > gpurun_out/r06b/amdsmi_static.json 2>&1; true)
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_multi.py tests/test_gpu_parallel.py > gpurun_out/r06b/gputests.txt 2>&1 &&
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r06b/bench.json 2> gpurun_out/r06b/bench.err
