#!/bin/bash
# Round 6: CRC table lookups at fixed LDS addresses (no per-lookup add; no __syncthreads_or
# static LDS) in the grouped row and tile kernels.  The GPU suite on the new library, then the
# chunk-CRC chains (c4crc / c3crc write, c3crc / c4crc read) and c4 / c3 writes, new against
# the previous library (libzarrhip_lab_old.so, the same sources at the previous commit),
# alternated, under rocprofv3 kernel traces.  Records → gpurun_out/r06ldsfold.
# (Lab records: the fixed-address form was reverted after these runs; summary.json holds the
# kernel times.  libzarrhip_lab_old.so was the committed sources built into a lab library.)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r06ldsfold
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R" || exit 1
timeout -k 10 800 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/gputests.out" 2> "$OUT/gputests.err"
rc=$?
echo "== gputests rc=$rc" >&2
tail -n 2 "$OUT/gputests.out" >&2
if [ $rc -ne 0 ]; then tail -n 40 "$OUT/gputests.out" >&2; exit $rc; fi
cd /tmp || exit 1
B="python3 $R/bench.py --no-cpu-baseline --no-extras --no-host-inclusive --allocations 1 --steps 3 --warmup 1"
for pass in 1 2; do
  for lib in new old; do
    if [ $lib = new ]; then unset ZH_LIB_PATH; else export ZH_LIB_PATH=$R/zarr-java_amd/zarrhip/libzarrhip_lab_old.so; fi
    for cfg in "write c4crc" "write c3crc" "read c3crc" "read c4crc" "write c3" "write c4"; do
      set -- $cfg
      D="$OUT/${pass}_${lib}_$1_$2"
      mkdir -p "$D"
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$D/trace" -o run -- $B --op $1 --config $2 > "$D/out" 2> "$D/err"
      rc=$?
      echo "== $D rc=$rc" >&2
      if [ $rc -ne 0 ]; then tail -n 40 "$D/err" >&2; exit $rc; fi
    done
  done
done
echo done >&2
