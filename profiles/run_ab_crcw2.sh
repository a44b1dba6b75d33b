#!/bin/bash
# chunk-CRC writes with the grouped kernels: c3crc (ZH_ENC_GROUP) and c4crc (ZH_ENC_TGROUP)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r02abcrcw2}
mkdir -p "$OUT"
run() {  # tag cfg env...
  local tag=$1 cfg=$2; shift 2
  env "$@" timeout -k 10 200 python3 "$R/bench.py" --op write --config $cfg --steps 5 --warmup 2 \
    --no-cpu-baseline --no-extras > "$OUT/$tag.json" 2> "$OUT/$tag.err" || exit $?
  echo "$tag $(python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(d['value'],d['ms_per_step'])" "$OUT/$tag.json")"
}
for rep in 1 2; do
  run c3crc_g2_$rep c3crc ZH_ENC_GROUP=2
  run c3crc_g1_$rep c3crc ZH_ENC_GROUP=1
  run c3crc_g4_$rep c3crc ZH_ENC_GROUP=4
  run c3crc_g0_$rep c3crc ZH_ENC_GROUP=0
  run c4crc_g2_$rep c4crc ZH_ENC_TGROUP=2
  run c4crc_g1_$rep c4crc ZH_ENC_TGROUP=1
done
