#!/bin/bash
# chunk-CRC writes: c4crc tile encode at 3 waves/SIMD vs unconstrained (ZH_CRC_W3), c3crc row
# encode with 4 vs 8 rows in flight per lane (ZH_ENC_DEEP)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r02abcrcw}
mkdir -p "$OUT"
run() {  # tag cfg env...
  local tag=$1 cfg=$2; shift 2
  env "$@" timeout -k 10 200 python3 "$R/bench.py" --op write --config $cfg --steps 5 --warmup 2 \
    --no-cpu-baseline --no-extras > "$OUT/$tag.json" 2> "$OUT/$tag.err" || exit $?
  echo "$tag $(python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(d['value'],d['ms_per_step'])" "$OUT/$tag.json")"
}
for rep in 1 2; do
  run c4crc_w3_$rep c4crc ZH_CRC_W3=1
  run c4crc_w2_$rep c4crc ZH_CRC_W3=0
  run c3crc_u8_$rep c3crc ZH_ENC_DEEP=1
  run c3crc_u4_$rep c3crc ZH_ENC_DEEP=0
done
