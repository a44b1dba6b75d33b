set -o pipefail
mkdir -p gpurun_out/r02c
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02c/gpu_tests.log 2>&1
