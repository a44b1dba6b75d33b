#!/bin/bash
# Round 3: cache policy of the chunk-CRC kernels: the new parity tests, the write A/B of
# cached payload stores (ZH_ENC_CRC_STNT=0) on c4crc and c3crc, the aligned tile encode
# (ZH_ENC_ALIGN=1), WRITE_SIZE with them.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03st
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
step tests 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_crc_tiles.py -k "cache_policy or chunk_groups or grouped_row_decode or tile_encode_chunk_crc or tile_groups or aligned" -x -q --timeout 120 --timeout-method thread
cd /tmp || exit 1
step ab_w_c4crc 600 python3 $R/profiles/ab_write_env.py c4crc 1 4 - ZH_ENC_CRC_STNT=0 ZH_ENC_ALIGN=1 ZH_ENC_ALIGN=1,ZH_ENC_ALIGN_PF=0
step ab_w_c3crc 600 python3 $R/profiles/ab_write_env.py c3crc 1 4 - ZH_ENC_CRC_STNT=0
B="python3 $R/bench.py --no-cpu-baseline --no-extras --no-host-inclusive --op write"
export ZH_ENC_ALIGN=1
step wwrite_c4crc_aligned 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/wwrite_c4crc_aligned" -o run -- $B --config c4crc --steps 2 --warmup 1
unset ZH_ENC_ALIGN
export ZH_ENC_CRC_STNT=0
step wwrite_c4crc_cached 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/wwrite_c4crc_cached" -o run -- $B --config c4crc --steps 2 --warmup 1
