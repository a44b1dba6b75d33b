#!/bin/bash
# grouped tile encode variants on c4 write: G (ZH_ENC_TGROUP)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r02abtenc}
mkdir -p "$OUT"
for rep in 1 2; do
  IFS=, read -ra VL <<< "${VARIANTS:-1,2,4,0}"
  for v in "${VL[@]}"; do
    set -- $v
    ZH_ENC_TGROUP=$1 timeout -k 10 200 python3 "$R/bench.py" --op write --config ${CFG:-c4} --steps 5 --warmup 2 \
      --no-cpu-baseline --no-extras > "$OUT/w_tg$1_$rep.json" 2> "$OUT/w_tg$1_$rep.err" || exit $?
    echo "TG=$1 rep=$rep $(python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(d['value'],d['ms_per_step'])" "$OUT/w_tg$1_$rep.json")"
  done
done
