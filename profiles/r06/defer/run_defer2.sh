#!/bin/bash
# Round 6: the c4crc tile encode folding each step's CRC under the next step's loads (DEFER,
# the build under test) against folding it right after the stores (libzarrhip_lab_nodefer.so,
# -DZH_LAB_DEFER=0): the CRC tile / write tests on the new build, then both alternated under
# rocprofv3 kernel traces (the fold inside the live branch; nodefer = the previous commit).
# Records → gpurun_out/r06defer2.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r06defer2
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R" || exit 1
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/tests.out" 2> "$OUT/tests.err"
rc=$?
echo "== tests rc=$rc" >&2
tail -n 2 "$OUT/tests.out" >&2
if [ $rc -ne 0 ]; then tail -n 40 "$OUT/tests.out" >&2; exit $rc; fi
cd /tmp || exit 1
B="python3 $R/bench.py --no-cpu-baseline --no-extras --no-host-inclusive --allocations 1 --steps 3 --warmup 1 --op write --config c4crc"
for pass in 1 2 3; do
  for lib in defer nodefer; do
    if [ $lib = defer ]; then unset ZH_LIB_PATH; else export ZH_LIB_PATH=$R/zarr-java_amd/zarrhip/libzarrhip_lab_$lib.so; fi
    D="$OUT/${pass}_$lib"
    mkdir -p "$D"
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$D/trace" -o run -- $B > "$D/out" 2> "$D/err"
    rc=$?
    echo "== $D rc=$rc" >&2
    if [ $rc -ne 0 ]; then tail -n 40 "$D/err" >&2; exit $rc; fi
  done
done
echo done >&2
