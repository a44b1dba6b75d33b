# A/B of the CRC-fused tile kernel, same box: previous binary (libzarrhip_head.so), the
# restructured kernel unconstrained (ZH_CRC_W3=0) and held to 3 waves (default)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r02crc
mkdir -p $O
for rep in 1 2; do
  ZH_LIB_PATH=$R/zarr-java_amd/zarrhip/libzarrhip_head.so timeout -k 10 200 python $R/bench.py --config c4crc --steps 10 --warmup 3 --no-cpu-baseline --no-extras > $O/head_$rep.json 2> $O/head_$rep.err || exit $?
  ZH_CRC_W3=0 timeout -k 10 200 python $R/bench.py --config c4crc --steps 10 --warmup 3 --no-cpu-baseline --no-extras > $O/w2_$rep.json 2> $O/w2_$rep.err || exit $?
  timeout -k 10 200 python $R/bench.py --config c4crc --steps 10 --warmup 3 --no-cpu-baseline --no-extras > $O/w3_$rep.json 2> $O/w3_$rep.err || exit $?
  timeout -k 10 200 python $R/bench.py --config c4 --steps 10 --warmup 3 --no-cpu-baseline --no-extras > $O/c4_$rep.json 2> $O/c4_$rep.err || exit $?
done
