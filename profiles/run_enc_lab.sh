set -o pipefail
mkdir -p gpurun_out/r02lab
timeout -k 10 300 zarr-java_amd/tools/enc_lab > gpurun_out/r02lab/enc_lab.json 2> gpurun_out/r02lab/enc_lab.err
