#!/bin/bash
# Round 6: the fixed-address CRC lookups with a workgroup barrier at each work item (product
# build) against the same without it (libzarrhip_lab_nosync.so, -DZH_LAB_ITEM_SYNC=0) and the
# previous library (libzarrhip_lab_old.so), alternated, kernel traces.  Records →
# gpurun_out/r06sync.
# (Lab records: the fixed-address form was reverted after these runs; summary.json holds the
# kernel times.  libzarrhip_lab_old.so was the committed sources built into a lab library.)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r06sync
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
B="python3 $R/bench.py --no-cpu-baseline --no-extras --no-host-inclusive --allocations 1 --steps 3 --warmup 1"
for pass in 1 2; do
  for lib in sync nosync old; do
    if [ $lib = sync ]; then unset ZH_LIB_PATH; else export ZH_LIB_PATH=$R/zarr-java_amd/zarrhip/libzarrhip_lab_$lib.so; fi
    for cfg in "write c4crc" "write c3crc" "read c3crc"; do
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
