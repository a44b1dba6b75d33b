#!/bin/bash
# Round 5: write-path encodes before the float all-fill change (libzarrhip_orig.so) vs after
# (libzarrhip.so), alternated in one call, per config.  Earlier calls: the masked compare in
# the CRC tile encode cost 2 % (c4crc 42.1 vs 43.0 ms) and a hoisted uniform branch 10 %
# (46.2 ms); the CRC tile encode now has kernels for each compare form.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05wab
mkdir -p "$OUT"
cd /tmp || exit 1
for cfg in ${WAB_CONFIGS:-c4crc c3crc c4}; do
  for i in 1 2 3; do
    for v in orig new; do
      lib=$R/zarr-java_amd/zarrhip/libzarrhip.so
      [ $v = orig ] && lib=$R/zarr-java_amd/zarrhip/libzarrhip_orig.so
      ZH_LIB_PATH=$lib timeout -k 10 200 python3 $R/bench.py --op write --config $cfg --no-cpu-baseline --no-extras --no-host-inclusive --steps 5 --warmup 2 > $OUT/${cfg}_${v}_$i.json 2> $OUT/${cfg}_${v}_$i.err || exit 1
      python3 -c "import json,sys; d=json.loads(open('$OUT/${cfg}_${v}_$i.json').read().strip().splitlines()[-1]); print('$cfg', '$v', $i, d['ms_per_step'])" >&2
    done
  done
done
echo done >&2
