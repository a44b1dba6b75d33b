#!/bin/bash
# Round 3: the aligned-window row-CRC decode (tiles_rowcrc_kernel ALN): the CRC tile tests,
# an interleaved A/B of ZH_DEC_ALIGN on c4crc, and FETCH_SIZE / WRITE_SIZE passes of the
# c4crc bench with the default (aligned) kernel.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03al
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  echo "== $name: $*" >&2
  timeout -k 10 "$t" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  echo "== $name rc=$rc" >&2
  if [ $rc -ne 0 ]; then exit $rc; fi
}
cd "$R" || exit 1
step tests 600 python -u -m pytest tests/test_gpu_crc_tiles.py -x -q --timeout 120 --timeout-method thread
cd /tmp || exit 1
step ab 600 python3 $R/profiles/ab_decode_env.py c4crc 1 6 - ZH_DEC_ALIGN=0
export ZH_DEC_ALIGN=1  # the profiles below: the aligned kernel
B="python3 $R/bench.py --no-cpu-baseline --no-extras --no-host-inclusive"
step trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- $B --config c4crc --steps 5 --warmup 2
step pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- $B --config c4crc --steps 2 --warmup 1
step pmc_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- $B --config c4crc --steps 2 --warmup 1
