#!/bin/bash
# tile encode with the next step's loads before this step's stores (ZH_ENC_TPF) vs without
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r02abtpf}
mkdir -p "$OUT"
for rep in 1 2 3; do
  for cfg in c4 c4crc; do
    for pf in 0 1; do
      ZH_ENC_TPF=$pf timeout -k 10 200 python3 "$R/bench.py" --op write --config $cfg --steps 5 --warmup 2 \
        --no-cpu-baseline --no-extras > "$OUT/w_${cfg}_pf${pf}_$rep.json" 2> "$OUT/w_${cfg}_pf${pf}_$rep.err" || exit $?
      echo "$cfg pf=$pf rep=$rep $(python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(d['value'],d['ms_per_step'])" "$OUT/w_${cfg}_pf${pf}_$rep.json")"
    done
  done
done
