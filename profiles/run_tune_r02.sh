set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r02tune
mkdir -p $O
TUNE_GRIDS=32,64,128,256,512 TUNE_NT=0,1,3 TUNE_VARIANTS=1 timeout -k 10 400 python $R/profiles/tune_grid.py c4 4 > $O/tune_c4.json 2> $O/tune_c4.err &&
TUNE_GRIDS=32,64,128,256,512 TUNE_NT=0,1,3 TUNE_VARIANTS=1 timeout -k 10 400 python $R/profiles/tune_grid.py c3 4 > $O/tune_c3.json 2> $O/tune_c3.err
