set -o pipefail
mkdir -p gpurun_out/r02lab
for mb in 1024 2; do
  ZH_SCATTER_MB=$mb timeout -k 10 300 python3 profiles/placement_pmc.py c4 8 2 mix > gpurun_out/r02lab/placement_mix_$mb.json 2> gpurun_out/r02lab/placement_mix_$mb.err || exit $?
done
