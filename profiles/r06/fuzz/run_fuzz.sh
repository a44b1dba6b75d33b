#!/bin/bash
# Round 6: the seeded searches on the final tree with new seeds — corrupt indexes (seeds 4-6,
# 200 trials each), 2000 random write + read codec chains, 300 random Array API cases — all
# against the oracle.  Records → gpurun_out/r06fuzz.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r06fuzz
mkdir -p "$OUT"
cd "$R" || exit 1
for seed in 4 5 6; do
  echo "== seed $seed" >&2
  ZH_FUZZ_SEED=$seed ZH_FUZZ_TRIALS=200 timeout -k 10 400 python3 -u -m pytest tests/test_gpu_fuzz_index.py -x -q --timeout 250 --timeout-method thread -p no:cacheprovider > "$OUT/seed$seed.log" 2>&1
  rc=$?
  tail -n 2 "$OUT/seed$seed.log" >&2
  if [ $rc -ne 0 ]; then tail -n 40 "$OUT/seed$seed.log" >&2; exit $rc; fi
done
echo "== write/read 2000" >&2
ZH_FUZZ_WCASES=2000 timeout -k 10 900 python3 -u -m pytest tests/test_fuzz_write.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/write_read_2000.log" 2>&1
rc=$?
tail -n 2 "$OUT/write_read_2000.log" >&2
if [ $rc -ne 0 ]; then tail -n 40 "$OUT/write_read_2000.log" >&2; exit $rc; fi
echo "== api 300" >&2
ZH_FUZZ_APICASES=300 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_api_fuzz.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/api_300.log" 2>&1
rc=$?
tail -n 2 "$OUT/api_300.log" >&2
if [ $rc -ne 0 ]; then tail -n 40 "$OUT/api_300.log" >&2; exit $rc; fi
echo done >&2
