#!/bin/bash
# Round 3: does the aligned-window kernel's LDS (54 436 B per workgroup) cost occupancy?  The
# unaligned row-CRC kernel padded to the same dynamic LDS (ZH_LDS_PAD) vs unpadded, and the
# aligned kernel, interleaved on c4crc.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03occ
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
timeout -k 10 600 python3 $R/profiles/ab_decode_env.py c4crc 1 6 - ZH_DEC_ALIGN=0 \
  ZH_DEC_ALIGN=0,ZH_LDS_PAD=160 > "$OUT/ab.out" 2> "$OUT/ab.err"
