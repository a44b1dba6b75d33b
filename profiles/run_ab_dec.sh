set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r02abdec
mkdir -p $O
timeout -k 10 200 python -u $R/profiles/ab_decode_env.py c3 1 3 ZH_DEC_RGROUP=0 ZH_DEC_RGROUP=8 > $O/c3.json 2> $O/c3.err &&
timeout -k 10 200 python -u $R/profiles/ab_decode_env.py c3nest 1 3 ZH_DEC_RGROUP=0 ZH_DEC_RGROUP=8 > $O/c3nest.json 2> $O/c3nest.err &&
timeout -k 10 200 python -u $R/profiles/ab_decode_env.py c4 1 3 ZH_DEC_TGROUP=4 ZH_DEC_TGROUP=8 ZH_DEC_TGROUP=2 > $O/c4.json 2> $O/c4.err
