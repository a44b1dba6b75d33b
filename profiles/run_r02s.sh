set -o pipefail
# Staging pool in the Python Array mirror: GPU tests of the mirror and the store-inclusive
# read (bench line), on a fresh box.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r02s
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_array.py tests/test_v2.py tests/test_http_store.py tests/test_reshape.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/array_tests.log 2>&1 &&
timeout -k 10 500 python $R/bench.py > $O/bench_n1.json 2> $O/bench_n1.err
