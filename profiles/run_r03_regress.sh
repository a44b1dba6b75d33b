#!/bin/bash
# Round 3: is the c4crc / c4 write (and decode) of the round-3 library slower than round 2's?
# The same A/B harness runs once per library (ZH_LIB_PATH: round 2's build, libzarrhip_r02.so,
# built from d1e6bcf), alternating, on one box.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03reg
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
step() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  echo "== $name: $*" >&2
  timeout -k 10 "$t" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  echo "== $name rc=$rc" >&2
  if [ $rc -ne 0 ]; then exit $rc; fi
}
for k in 1 2; do
  for lib in r03 r02; do
    if [ $lib = r02 ]; then export ZH_LIB_PATH=$R/zarr-java_amd/zarrhip/libzarrhip_r02.so; else unset ZH_LIB_PATH; fi
    step w_c4crc_${lib}_$k 300 python3 $R/profiles/ab_write_env.py c4crc 1 4 -
    step w_c4_${lib}_$k 300 python3 $R/profiles/ab_write_env.py c4 1 4 -
    step d_c4crc_${lib}_$k 300 python3 $R/profiles/ab_decode_env.py c4crc 1 4 -
  done
done
unset ZH_LIB_PATH
