#!/bin/bash
# Round 6 lab: the c4crc tile encode with its next step's loads issued before the CRC (PF, lab_pf.patch,
# -DZH_LAB_PF=true) against the product (loads at the step start), alternated; kernel traces.
# Records → gpurun_out/r06pf.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r06pf
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
W="python3 $R/bench.py --no-cpu-baseline --no-extras --no-host-inclusive --op write --config c4crc --steps 3 --warmup 1"
i=0
for lib in product pf product pf; do
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
echo done >&2
