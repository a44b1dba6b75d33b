set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r02f
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 &&
timeout -k 10 300 python $R/bench.py --config c2 --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_c2.json 2> $O/bench_c2.err &&
timeout -k 10 300 python $R/bench.py --config c4crc --steps 10 --warmup 3 --no-cpu-baseline --no-extras > $O/bench_c4crc.json 2> $O/bench_c4crc.err &&
timeout -k 10 300 python $R/bench.py --config c4crc --op write --steps 5 --warmup 2 > $O/bench_c4crc_write.json 2> $O/bench_c4crc_write.err &&
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_c2 -o run -- python3 $R/bench.py --config c2 --steps 5 --warmup 2 --no-cpu-baseline --no-extras > $O/trace_c2.out 2> $O/trace_c2.err
