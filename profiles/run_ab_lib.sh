#!/bin/bash
# the same bench command against two library builds, interleaved (ZH_LIB_PATH)
#   CMD="--op write --config c4crc" profiles/run_ab_lib.sh tag other.so
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r02ablib}
OTHER=${2:-$R/zarr-java_amd/zarrhip/libzarrhip_old.so}
mkdir -p "$OUT"
for rep in 1 2 3; do
  for lib in cur other; do
    if [ $lib = other ]; then export ZH_LIB_PATH=$OTHER; else unset ZH_LIB_PATH; fi
    timeout -k 10 200 python3 "$R/bench.py" ${CMD:---config c4} --steps 5 --warmup 2 --no-cpu-baseline --no-extras \
      > "$OUT/${lib}_$rep.json" 2> "$OUT/${lib}_$rep.err" || exit $?
    echo "$lib rep=$rep $(python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(d['value'],d['ms_per_step'])" "$OUT/${lib}_$rep.json")"
  done
done
