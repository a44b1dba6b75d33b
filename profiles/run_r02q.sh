set -o pipefail
# c4 tile groups G = 8 with the prefetching form vs G = 4; the 2-rank strong rehearsal (arena
# pair per rank); then the round-2 profiles (run_r02_profile2.sh).
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r02q
mkdir -p $O
timeout -k 10 200 python -u $R/profiles/ab_decode_env.py c4 1 3 ZH_DEC_TGROUP=4 ZH_DEC_TGROUP=8 > $O/ab_c4_g8pf.json 2> $O/ab_c4_g8pf.err &&
timeout -k 10 300 python -u $R/bench.py --gpus 2 --ydiv 4 --steps 10 --warmup 2 > $O/bench_n2_rehearsal.json 2> $O/bench_n2_rehearsal.err &&
bash $R/profiles/run_r02_profile2.sh
