#!/bin/bash
# Tile-kernel CRC parity tests, then an interleaved A/B of c4crc with the data-byte CRC
# lookups from the 256-entry byte tables (ZH_CRC_NIB=0) or from conflict-free 16-entry nibble
# tables (ZH_CRC_NIB=1).  GPU box, repo root.
# The ZH_CRC_NIB variant was removed after this run measured it 55 % slower
# (profiles/r01/experiments/crc_nib/); the script is kept as the record of the experiment.
set -u
O=gpurun_out/nib
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_crc_tiles.py tests/test_gpu_parity.py -x -q \
  --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for gl in 0 1; do
    ZH_CRC_NIB=$gl timeout -k 10 200 python3 bench.py --config c4crc --steps 5 --warmup 2 \
      --no-cpu-baseline > $O/c4crc_nib${gl}_$r.json 2> $O/c4crc_nib${gl}_$r.err || exit 2
    python3 -c "import json;d=json.load(open('$O/c4crc_nib${gl}_$r.json'));print('nib=$gl r=$r',d['value'],d['ms_per_step'],d['roofline']['kernel_ms'])"
  done
done
cd /tmp || exit 3
export TMPDIR=/tmp
ZH_CRC_NIB=1 timeout -k 10 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES \
  --output-format csv -d "$GRAFT_REPO_ROOT/$O/lds_nib" -o run -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --config c4crc --steps 1 --warmup 1 --no-cpu-baseline \
  > "$GRAFT_REPO_ROOT/$O/lds_nib.out" 2> "$GRAFT_REPO_ROOT/$O/lds_nib.err" || exit 4
echo lds_nib ok
