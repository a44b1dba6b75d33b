set -o pipefail
# Re-entry check of the committed tree on a fresh box: the whole GPU suite, smoke, the
# default bench line.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r02t
mkdir -p $O
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 400 python $R/bench.py > $O/bench_n1.json 2> $O/bench_n1.err
