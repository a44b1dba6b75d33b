#!/bin/bash
# Round 5: ZH_IDX_CRC_FUSE at full size, interleaved in one process (kernel window and wall time
# per step), c4 at half y over three output placements, c3 full.  Records → gpurun_out/r05fuse2.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05fuse2
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  echo "== $name: $*" >&2
  timeout -k 10 "$t" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  echo "== $name rc=$rc" >&2
  if [ $rc -ne 0 ]; then tail -n 60 "$OUT/$name.out" "$OUT/$name.err" >&2; exit $rc; fi
}
cd "$R" || exit 1
step tests 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread
export AB_OUTS=3 AB_YDIV=2
step ab_c4 400 python3 profiles/r05/env_ab.py "$OUT/fuse_c4.json" c4 5 10 ZH_IDX_CRC_FUSE=1 ZH_IDX_CRC_FUSE=0
export AB_OUTS=1 AB_YDIV=1
step ab_c3 300 python3 profiles/r05/env_ab.py "$OUT/fuse_c3.json" c3 5 10 ZH_IDX_CRC_FUSE=1 ZH_IDX_CRC_FUSE=0
echo done >&2
