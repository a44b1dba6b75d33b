set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r02abwr
mkdir -p $O
timeout -k 10 200 python -u $R/profiles/ab_write_env.py c3 4 3 ZH_ENC_XPOSE=0 ZH_ENC_XPOSE=1 ZH_ENC_XPOSE=1,ZH_ITEM_PERM=0 ZH_ENC_XPOSE=0,ZH_ITEM_PERM=0 > $O/c3.json 2> $O/c3.err &&
timeout -k 10 200 python -u $R/profiles/ab_write_env.py c4 4 3 - ZH_ITEM_PERM=0 ZH_ENC_TGROUP=4 ZH_ENC_TGROUP=4,ZH_ITEM_PERM=0 > $O/c4.json 2> $O/c4.err &&
timeout -k 10 300 python $R/bench.py --op write --config c3 --steps 5 --warmup 2 --no-cpu-baseline --no-extras > $O/write_c3.json 2> $O/write_c3.err &&
timeout -k 10 300 python $R/bench.py --op write --config c4 --steps 5 --warmup 2 --no-cpu-baseline --no-extras > $O/write_c4.json 2> $O/write_c4.err
