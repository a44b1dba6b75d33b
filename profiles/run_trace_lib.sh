#!/bin/bash
# kernel trace of one bench command against the current and another library build
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r02tlib}
OTHER=${2:-$R/zarr-java_amd/zarrhip/libzarrhip_old.so}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
for lib in cur other; do
  if [ $lib = other ]; then export ZH_LIB_PATH=$OTHER; else unset ZH_LIB_PATH; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$lib" -o run -- \
    python3 "$R/bench.py" ${CMD:---config c4} --steps 5 --warmup 2 --no-cpu-baseline --no-extras \
    > "$OUT/$lib.out" 2> "$OUT/$lib.err" || exit $?
done
