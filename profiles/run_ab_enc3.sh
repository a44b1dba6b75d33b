#!/bin/bash
# grouped encode variants on c3 write: G (ZH_ENC_GROUP) x U (ZH_ENC_GU rows in flight per lane)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r02abenc3}
mkdir -p "$OUT"
for rep in 1 2; do
  IFS=, read -ra VL <<< "${VARIANTS:-1 2,1 4,1 8,2 2,2 4,2 8,4 2,0 4}"
  for v in "${VL[@]}"; do
    set -- $v
    ZH_ENC_GROUP=$1 ZH_ENC_GU=$2 timeout -k 10 200 python3 "$R/bench.py" --op write --config c3 --steps 5 --warmup 2 \
      --no-cpu-baseline --no-extras > "$OUT/w_g$1_u$2_$rep.json" 2> "$OUT/w_g$1_u$2_$rep.err" || exit $?
    echo "G=$1 U=$2 rep=$rep $(python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(d['value'],d['ms_per_step'])" "$OUT/w_g$1_u$2_$rep.json")"
  done
done
