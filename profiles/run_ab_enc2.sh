#!/bin/bash
# grouped encode variants on c3 write: G (ZH_ENC_GROUP) x U (ZH_ENC_DEEP=2 → 8 rows per lane)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r02abenc2}
mkdir -p "$OUT"
for rep in 1 2; do
  for v in "4 1" "4 2" "8 1" "8 2" "2 1" "0 1"; do
    set -- $v
    ZH_ENC_GROUP=$1 ZH_ENC_DEEP=$2 timeout -k 10 200 python3 "$R/bench.py" --op write --config c3 --steps 5 --warmup 2 \
      --no-cpu-baseline --no-extras > "$OUT/w_g$1_d$2_$rep.json" 2> "$OUT/w_g$1_d$2_$rep.err" || exit $?
    echo "G=$1 deep=$2 rep=$rep $(python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(d['value'],d['ms_per_step'])" "$OUT/w_g$1_d$2_$rep.json")"
  done
done
