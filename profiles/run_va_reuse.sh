set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r02va
mkdir -p $O
for args in "plain 2 2 5" "view 2 2 5" "plain 1024 2 5" "view 1024 2 5" "plain 2 8 3" "view 2 8 3"; do
  timeout -k 10 60 python -u $R/profiles/va_reuse_lab.py $args >> $O/va.jsonl 2>> $O/va.err || exit $?
done
for args in "view 2 2 5" "plain 2 2 5"; do
  ZH_SCATTER_RETIRE=1 timeout -k 10 60 python -u $R/profiles/va_reuse_lab.py $args >> $O/va.jsonl 2>> $O/va.err || exit $?
done
timeout -k 10 120 python -u -m pytest tests/test_gpu_alloc.py -x -q --timeout 60 --timeout-method thread > $O/alloc_tests.log 2>&1 &&
timeout -k 10 300 python -u $R/profiles/ab_xpose.py c3 3 > $O/ab_xpose_c3.json 2> $O/ab_xpose_c3.err
