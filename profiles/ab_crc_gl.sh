#!/bin/bash
# Tile-kernel CRC parity tests, then an interleaved A/B of c4crc with the hi-word CRC lookups
# from the LDS (ZH_CRC_GL=0) or through the vector L1 (ZH_CRC_GL=1).  GPU box, repo root.
# The ZH_CRC_GL variant was removed after this run measured it 44 % slower
# (profiles/r01/experiments/crc_gl/); the script is kept as the record of the experiment.
set -u
O=gpurun_out/gl
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_crc_tiles.py tests/test_gpu_parity.py -x -q \
  --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for gl in 0 1; do
    ZH_CRC_GL=$gl timeout -k 10 200 python3 bench.py --config c4crc --steps 5 --warmup 2 \
      --no-cpu-baseline > $O/c4crc_gl${gl}_$r.json 2> $O/c4crc_gl${gl}_$r.err || exit 2
    python3 -c "import json;d=json.load(open('$O/c4crc_gl${gl}_$r.json'));print('gl=$gl r=$r',d['value'],d['ms_per_step'],d['roofline']['kernel_ms'])"
  done
done
