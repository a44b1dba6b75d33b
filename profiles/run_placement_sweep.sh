set -o pipefail
mkdir -p gpurun_out/r02lab
for mb in 16 64 256 1024 4096; do
  ZH_SCATTER_MB=$mb timeout -k 10 300 python3 profiles/placement_pmc.py c4 6 2 scatter > gpurun_out/r02lab/placement_sweep_$mb.json 2> gpurun_out/r02lab/placement_sweep_$mb.err || exit $?
done
timeout -k 10 300 python3 profiles/placement_pmc.py c4 6 2 plain > gpurun_out/r02lab/placement_sweep_plain.json 2> gpurun_out/r02lab/placement_sweep_plain.err
