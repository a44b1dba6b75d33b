#!/bin/bash
# Round 5: a wider corrupt-index search (tests/test_gpu_fuzz_index.py) over several seeds.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05fuzz
mkdir -p "$OUT"
cd "$R" || exit 1
for seed in 1 2 3 4 5 6; do
  echo "== seed $seed" >&2
  ZH_FUZZ_SEED=$seed ZH_FUZZ_TRIALS=200 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_fuzz_index.py -x -q --timeout 250 --timeout-method thread -p no:cacheprovider > "$OUT/seed$seed.log" 2>&1
  rc=$?
  tail -n 3 "$OUT/seed$seed.log" >&2
  if [ $rc -ne 0 ]; then tail -n 40 "$OUT/seed$seed.log" >&2; exit $rc; fi
done
echo done >&2
