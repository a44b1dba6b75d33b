#!/bin/bash
# Round 4 A/B: the 16-tile encode (ZH_ENC_T16 = G: G chunks per work item, 16/G tiles of each
# per step, 512 threads, 512-B region reads and 512-B payload rows at G = 4) against the default
# 8-tile grouped encode (G = 2), c4 write, full array, every output size checked; its parity
# cases first.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04f
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
step t16_tests 300 python3 -u -m pytest "tests/test_gpu_parity.py::test_device_encode_tiles16" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step abw_c4 500 python3 profiles/ab_write_env.py c4 1 3 - ZH_ENC_T16=4 ZH_ENC_T16=2 ZH_ENC_T16=8 ZH_ENC_T16=4,ZH_ITEM_ROW=4 ZH_ENC_T16=1
step abw_c4q 300 python3 profiles/ab_write_env.py c4 4 3 - ZH_ENC_T16=4 ZH_ENC_T16=2
echo done >&2
