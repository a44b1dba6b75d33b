#!/bin/bash
# Round 5: the seeded searches again on the last tree, both small-plan forms (ZH_SMALL_ONE 0/1
# parametrized in the tests): corrupt indexes over three seeds at 200 trials, 1000 random write
# + read chains.  Records → gpurun_out/r05fuzz2.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05fuzz2
mkdir -p "$OUT"
cd "$R" || exit 1
for seed in 1 2 3; do
  echo "== seed $seed" >&2
  ZH_FUZZ_SEED=$seed ZH_FUZZ_TRIALS=200 timeout -k 10 400 python3 -u -m pytest tests/test_gpu_fuzz_index.py -x -q --timeout 250 --timeout-method thread -p no:cacheprovider > "$OUT/seed$seed.log" 2>&1
  rc=$?
  tail -n 3 "$OUT/seed$seed.log" >&2
  if [ $rc -ne 0 ]; then tail -n 40 "$OUT/seed$seed.log" >&2; exit $rc; fi
done
echo "== write/read 1000" >&2
ZH_FUZZ_WCASES=1000 timeout -k 10 600 python3 -u -m pytest tests/test_fuzz_write.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "read_random_regions or device_write" > "$OUT/write_read_1000.log" 2>&1
rc=$?
tail -n 3 "$OUT/write_read_1000.log" >&2
if [ $rc -ne 0 ]; then tail -n 40 "$OUT/write_read_1000.log" >&2; exit $rc; fi
echo done >&2
