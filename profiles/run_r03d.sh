set -o pipefail
mkdir -p gpurun_out/r03d
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03d/pytest.log 2>&1 && \
bash profiles/run_r03_regress.sh && \
timeout -k 10 600 python -u bench.py > gpurun_out/r03d/bench.json 2> gpurun_out/r03d/bench.err
