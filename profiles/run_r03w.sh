#!/bin/bash
# Round 3 last check of the committed tree: all GPU tests and smoke.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03w
mkdir -p "$OUT"
cd "$R" || exit 1
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 170 --timeout-method thread > "$OUT/pytest.out" 2> "$OUT/pytest.err" && \
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.out" 2> "$OUT/smoke.err"
