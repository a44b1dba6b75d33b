set -o pipefail
mkdir -p gpurun_out/r02lab
timeout -k 10 200 zarr-java_amd/tools/chunk_lab 1024 160 > gpurun_out/r02lab/chunk_lab_1g.json 2> gpurun_out/r02lab/chunk_lab_1g.err &&
timeout -k 10 200 zarr-java_amd/tools/chunk_lab 256 400 > gpurun_out/r02lab/chunk_lab_256m.json 2> gpurun_out/r02lab/chunk_lab_256m.err
