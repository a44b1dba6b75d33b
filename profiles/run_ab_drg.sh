#!/bin/bash
# tile decode over G chunks per work item (ZH_DEC_RGROUP) vs the default, interleaved, c4
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r02abdrg}
mkdir -p "$OUT"
for rep in 1 2 3; do
  IFS=, read -ra VL <<< "${VARIANTS:-0,2,4,1}"
  for v in "${VL[@]}"; do
    ZH_DEC_RGROUP=$v timeout -k 10 200 python3 "$R/bench.py" --config ${CFG:-c4} --steps 20 --warmup 3 \
      --no-cpu-baseline --no-extras > "$OUT/d_tg${v}_$rep.json" 2> "$OUT/d_tg${v}_$rep.err" || exit $?
    echo "DTG=$v rep=$rep $(python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(d['value'],d['ms_per_step'])" "$OUT/d_tg${v}_$rep.json")"
  done
done
