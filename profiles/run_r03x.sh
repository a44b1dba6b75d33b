#!/bin/bash
# Round 3: c4crc write vs the grid of the fused tile encode (ZH_BLOCKS_PER_CU: workgroups per
# CU of the grid-stride kernels; default 256, i.e. one work item per workgroup here).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03x
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
timeout -k 10 600 python3 $R/profiles/ab_write_env.py c4crc 1 3 - ZH_BLOCKS_PER_CU=3 ZH_BLOCKS_PER_CU=6 ZH_BLOCKS_PER_CU=24 > "$OUT/ab.out" 2> "$OUT/ab.err"
