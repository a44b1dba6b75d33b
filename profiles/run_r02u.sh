set -o pipefail
# CRC over LDS rows (tiles_rowcrc_kernel) and CRC waves (tiles_crcw_kernel): parity tests, an
# interleaved full-size c4crc A/B against the fused grouped kernel (default), and an occupancy
# lab on plain c4 (extra LDS per block: 4 -> 3 blocks per CU).
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUTD:-r02u}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_crc_tiles.py -k "crc_waves or grouped_tile" -m gpu -x -q --timeout 120 --timeout-method thread > $O/crc_tests.log 2>&1 &&
timeout -k 10 400 python -u $R/profiles/ab_decode_env.py c4crc 1 5 - ${CRC_VARIANTS:-ZH_DEC_CRCW=3,ZH_DEC_TGROUP=2 ZH_DEC_CRCW=3,ZH_DEC_TGROUP=1 ZH_DEC_CRCW=3,ZH_DEC_TGROUP=4} > $O/ab_crcw.json 2> $O/ab_crcw.err
