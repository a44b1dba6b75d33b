set -o pipefail
mkdir -p gpurun_out/r02lab
timeout -k 10 300 zarr-java_amd/tools/place_lab 6 > gpurun_out/r02lab/place_lab.json 2> gpurun_out/r02lab/place_lab.err
