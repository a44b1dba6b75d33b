#!/bin/bash
# Round 4 A/B: the grouped kernels' visit order over runs of R consecutive groups (ZH_ITEM_ROW =
# R; z-adjacent chunks read by workgroups running at once) against the golden-ratio order of
# single groups, interleaved in one process per config, every output verified: the write path
# (c4, c3, c4crc, c3crc: scattered region reads) and the decode (c4, c3, c4crc).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04e
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  echo "== $name: $*" >&2
  timeout -k 10 "$t" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  echo "== $name rc=$rc" >&2
  if [ $rc -ne 0 ]; then tail -n 40 "$OUT/$name.out" "$OUT/$name.err" >&2; exit $rc; fi
}
cd "$R" || exit 1
step smoke_tests 300 python3 -u -m pytest tests/test_gpu_crc_tiles.py tests/test_gpu_c2.py "tests/test_gpu_parity.py::test_item_row_order" "tests/test_gpu_parity.py::test_device_encode_tile_groups" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step abw_c4 500 python3 profiles/ab_write_env.py c4 1 3 - ZH_ITEM_ROW=4 ZH_ITEM_ROW=8 ZH_ITEM_ROW=16 ZH_ENC_TGROUP=8 ZH_ENC_TGROUP=8,ZH_ITEM_ROW=2 ZH_ENC_TGROUP=4,ZH_ITEM_ROW=4
step abw_c3 500 python3 profiles/ab_write_env.py c3 1 3 - ZH_ITEM_ROW=4 ZH_ITEM_ROW=8 ZH_ITEM_ROW=16 ZH_ENC_GROUP=4,ZH_ITEM_ROW=4
for cfg in c4crc c3crc; do
  step abw_$cfg 500 python3 profiles/ab_write_env.py $cfg 1 3 - ZH_ITEM_ROW=4 ZH_ITEM_ROW=8 ZH_ITEM_ROW=16
done
for cfg in c4 c3 c4crc; do
  step abd_$cfg 500 python3 profiles/ab_decode_env.py $cfg 1 3 - ZH_ITEM_ROW=2 ZH_ITEM_ROW=4 ZH_ITEM_ROW=8
done
echo done >&2
