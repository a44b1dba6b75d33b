#!/bin/bash
# Round 6 lab (DESIGN §4 "The chunk-CRC encode"): where the aligned CRC tile encode's time goes.
# Libraries (make lab LAB=…): aln0 = the product (the unaligned kernel), aln1 = aligned stores,
# aln2 = aligned without the slot 0-1 stores, aln3 = unaligned stores plus the slot 0-1 work.
# (When this ran, the default library was the aligned one and aln0 a lab build; the library
# roles are swapped here to match the tree since, the kernels are the same.)
# aln2/aln3 write wrong payloads, so their bench run ends in the write round-trip failure
# (exit 1) after the timed steps: that exit is expected, anything else stops the script.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r06aln
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
W="python3 $R/bench.py --no-cpu-baseline --no-extras --no-host-inclusive --op write --config c4crc --steps 3 --warmup 1"
i=0
for lib in 1 0 2 3 0 1; do
  i=$((i + 1))
  if [ $lib = 0 ]; then unset ZH_LIB_PATH; else export ZH_LIB_PATH=$R/zarr-java_amd/zarrhip/libzarrhip_lab_aln$lib.so; fi
  D="$OUT/${i}_aln$lib"
  mkdir -p "$D"
  echo "== $D" >&2
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$D/wtrace" -o run -- $W > "$D/out" 2> "$D/err"
  rc=$?
  echo "== rc=$rc" >&2
  if [ $rc -ne 0 ] && ! { [ $rc -eq 1 ] && [ $lib -ge 2 ]; }; then tail -n 40 "$D/err" >&2; exit $rc; fi
done
echo done >&2
