set -o pipefail
# Re-verification of the rebuilt tree: smoke, the whole GPU suite, the default bench line.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r02m
mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 &&
timeout -k 10 500 python $R/bench.py > $O/bench_n1.json 2> $O/bench_n1.err
