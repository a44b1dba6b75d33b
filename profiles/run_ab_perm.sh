set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r02abperm
mkdir -p $O
timeout -k 10 200 python -u $R/profiles/ab_decode_env.py c3 1 3 ZH_ITEM_PERM=0 ZH_ITEM_PERM=1 > $O/c3.json 2> $O/c3.err &&
timeout -k 10 200 python -u $R/profiles/ab_decode_env.py c4 1 3 ZH_ITEM_PERM=1 ZH_ITEM_PERM=0 > $O/c4.json 2> $O/c4.err
