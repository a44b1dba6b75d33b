#!/bin/bash
# Round 6: the c4crc tile encode with two sub-groups per workgroup sharing one set of CRC
# tables (4 waves per SIMD, the product) against one sub-group (3 per SIMD, make lab_sg1):
# first the GPU suite on the product, then both alternated under rocprofv3 kernel
# traces, then the product's PMC write / fetch passes.  Records → gpurun_out/r06sg.
# (The two-sub-group kernel was the product build when this ran; it measured slower and was
# removed, so this script no longer reproduces that arm.)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r06sg
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R" || exit 1
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/tests.out" 2> "$OUT/tests.err"
rc=$?
echo "== tests rc=$rc" >&2
if [ $rc -ne 0 ]; then tail -n 40 "$OUT/tests.out" >&2; exit $rc; fi
cd /tmp || exit 1
W="python3 $R/bench.py --no-cpu-baseline --no-extras --no-host-inclusive --op write --config c4crc --steps 3 --warmup 1"
i=0
for lib in product sg1 product sg1; do
  i=$((i + 1))
  if [ $lib = product ]; then unset ZH_LIB_PATH; else export ZH_LIB_PATH=$R/zarr-java_amd/zarrhip/libzarrhip_lab_$lib.so; fi
  D="$OUT/${i}_$lib"
  mkdir -p "$D"
  echo "== $D" >&2
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$D/wtrace" -o run -- $W > "$D/out" 2> "$D/err"
  rc=$?
  echo "== rc=$rc" >&2
  if [ $rc -ne 0 ]; then tail -n 40 "$D/err" >&2; exit $rc; fi
done
unset ZH_LIB_PATH
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/wfetch_c4crc" -o run -- $W > "$OUT/wfetch.out" 2> "$OUT/wfetch.err" || exit $?
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/wwrite_c4crc" -o run -- $W > "$OUT/wwrite.out" 2> "$OUT/wwrite.err" || exit $?
cp -r "$OUT/1_product/wtrace" "$OUT/wtrace_c4crc"
timeout -k 10 60 python3 $R/profiles/pmc_summary_write.py "$OUT" c4crc "$OUT/write_c4crc_summary.json" 206161575936 || exit $?
echo done >&2
