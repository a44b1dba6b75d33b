#!/bin/bash
# Round 3: the chunk-CRC kernels with the edge vectors of each contiguous payload segment
# loaded (decode, ZH_CRC_EDGE=1) or stored (encode, ZH_ENC_CRC_EDGE=1) temporal, against the
# default: interleaved A/B of the kernel time in one process, then FETCH_SIZE / WRITE_SIZE
# passes of each decode variant (c4crc, c3crc).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03crc
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
for cfg in c4crc c3crc; do
  step ab_$cfg 300 python3 $R/profiles/ab_decode_env.py $cfg 1 6 - ZH_CRC_EDGE=1
  step abw_$cfg 300 python3 $R/profiles/ab_write_env.py $cfg 1 6 - ZH_ENC_CRC_EDGE=1
done
B="python3 $R/bench.py --no-cpu-baseline --no-extras --no-host-inclusive"
for cfg in c4crc c3crc; do
  for e in 0 1; do
    export ZH_CRC_EDGE=$e
    step pmc_fetch_${cfg}_e$e 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch_${cfg}_e$e" -o run -- $B --config $cfg --steps 2 --warmup 1
  done
done
unset ZH_CRC_EDGE
