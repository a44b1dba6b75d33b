#!/bin/bash
# GPU parity tests + bench matrix (configs x env knobs).  usage: run_bench_matrix.sh TAG
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-exp}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R" || exit 1
timeout -k 10 600 python3 -m pytest tests -m gpu -q -x > "$OUT/gpu_tests.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/gpu_tests.log"
if [ $rc -ne 0 ]; then exit $rc; fi
run() {  # name env... -- args
  local name=$1; shift
  timeout -k 10 300 env "$@" > "$OUT/$name.json" 2> "$OUT/$name.err"
  local rc=$?
  echo "$name rc=$rc $(python3 -c "import json,sys;d=json.load(open('$OUT/$name.json'));print(d['value'],d['ms_per_step'],d['roofline']['kernel_ms'],d['roofline']['frac'])" 2>/dev/null)"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/$name.err"; exit $rc; fi
}
shift
for spec in "$@"; do
  # spec: name:config:ENV=VAL,ENV=VAL
  IFS=: read -r name cfg envs <<< "$spec"
  envargs=()
  if [ -n "$envs" ]; then IFS=, read -ra envargs <<< "$envs"; fi
  run "$name" "${envargs[@]}" python3 bench.py --config "$cfg" --steps 5 --warmup 2 --no-cpu-baseline
done
