#!/bin/bash
# write-path A/B: grouped encode (default) vs ZH_ENC_GROUP=0, interleaved, c3 and c2 and c3nest
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r02abenc}
mkdir -p "$OUT"
for rep in 1 2; do
  for g in -1 0; do
    for cfg in c3 c2 c3nest; do
      ZH_ENC_GROUP=$g timeout -k 10 200 python3 "$R/bench.py" --op write --config $cfg --steps 5 --warmup 2 \
        --no-cpu-baseline --no-extras > "$OUT/w_${cfg}_g${g}_$rep.json" 2> "$OUT/w_${cfg}_g${g}_$rep.err" || exit $?
      echo "$cfg g=$g rep=$rep $(python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(d['value'],d['ms_per_step'])" "$OUT/w_${cfg}_g${g}_$rep.json")"
    done
  done
done
