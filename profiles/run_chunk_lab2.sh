set -o pipefail
mkdir -p gpurun_out/r02lab
timeout -k 10 300 zarr-java_amd/tools/chunk_lab b 4 > gpurun_out/r02lab/chunk_lab_buffers.json 2> gpurun_out/r02lab/chunk_lab_buffers.err
