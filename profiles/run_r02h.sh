set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r02h
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "array or partial or stage or v2 or zstd" > $O/gpu_tests.log 2>&1
