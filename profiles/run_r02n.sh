set -o pipefail
# Placement lab (physical chunks vs chunk order vs virtual range), allocator tests, then
# re-verification of the rebuilt tree.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r02n
mkdir -p $O
timeout -k 10 120 python -u -m pytest tests/test_gpu_alloc.py -x -q --timeout 60 --timeout-method thread > $O/alloc_tests.log 2>&1 &&
timeout -k 10 240 python -u $R/profiles/placement_calib.py 8 3 > $O/calib2.jsonl 2> $O/calib2.err &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 &&
timeout -k 10 500 python $R/bench.py > $O/bench_n1.json 2> $O/bench_n1.err
