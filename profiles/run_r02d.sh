set -o pipefail
mkdir -p gpurun_out/r02d
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "array or blosc or zstd or v2" > gpurun_out/r02d/gpu_tests.log 2>&1
