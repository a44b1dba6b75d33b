#!/bin/bash
# Round 6 lab: the c4crc tile encode with each step's payload stores also deferred to the next
# step's load phase (-DZH_LAB_DEFER_ST=1, libzarrhip_lab_defst.so) against the product (stores
# right after the LDS reads, CRC deferred); the CRC tests on the lab build, then alternated
# kernel traces (kd0 = the product).  Records → gpurun_out/r06defst.
# (Lab record: slower, not kept; ZH_LAB_DEFER_ST is no longer in the source.)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r06defst
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R" || exit 1
ZH_LIB_PATH=$R/zarr-java_amd/zarrhip/libzarrhip_lab_defst.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_crc_tiles.py tests/test_fuzz_write.py tests/test_float_fill.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/tests_defst.out" 2> "$OUT/tests_defst.err"
rc=$?
echo "== tests rc=$rc" >&2
tail -n 2 "$OUT/tests_defst.out" >&2
if [ $rc -ne 0 ]; then tail -n 40 "$OUT/tests_defst.out" >&2; exit $rc; fi
cd /tmp || exit 1
B="python3 $R/bench.py --no-cpu-baseline --no-extras --no-host-inclusive --allocations 1 --steps 3 --warmup 1 --op write --config c4crc"
for pass in 1 2 3; do
  for lib in kd0 defst; do
    if [ $lib = kd0 ]; then unset ZH_LIB_PATH; else export ZH_LIB_PATH=$R/zarr-java_amd/zarrhip/libzarrhip_lab_$lib.so; fi
    D="$OUT/${pass}_$lib"
    mkdir -p "$D"
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$D/trace" -o run -- $B > "$D/out" 2> "$D/err"
    rc=$?
    echo "== $D rc=$rc" >&2
    if [ $rc -ne 0 ]; then tail -n 40 "$D/err" >&2; exit $rc; fi
  done
done
echo done >&2
