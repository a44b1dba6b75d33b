#!/bin/bash
# Round 6 lab: how much does the c4crc tile encode depend on workgroups per CU?  The product
# (3 per CU, LDS-bound) against the lab build padded to 2 per CU (make lab_pad PAD=25600),
# alternated, kernel time from rocprofv3 kernel traces.  Records → gpurun_out/r06occ.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r06occ
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
W="python3 $R/bench.py --no-cpu-baseline --no-extras --no-host-inclusive --op write --config c4crc --steps 3 --warmup 1"
i=0
for lib in product pad25600 product pad25600; do
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
