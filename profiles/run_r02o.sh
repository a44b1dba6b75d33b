set -o pipefail
# Fresh-range allocator (no virtual range mapped twice), lane-exchange row decode as the c3
# default, the faster-of-two arenas in the bench: VA lab, allocator + parity tests, full GPU
# suite, bench.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r02o
mkdir -p $O
for args in "plain 2 8 3" "view 2 8 3" "view 1024 2 5" "plain 2 2 5"; do
  timeout -k 10 60 python -u $R/profiles/va_reuse_lab.py $args >> $O/va.jsonl 2>> $O/va.err || exit $?
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_alloc.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "alloc or lane_exchange or grouped_row or chunk_groups" > $O/xpose_tests.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 &&
timeout -k 10 500 python $R/bench.py > $O/bench_n1.json 2> $O/bench_n1.err
