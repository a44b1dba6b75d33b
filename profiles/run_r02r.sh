set -o pipefail
# Round-2 final-state bench on a fresh box: default bench line (c4 headline + extras), then
# the write path and the chunk-CRC decode configs with the arena pair.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r02r_${1:-a}
mkdir -p $O
timeout -k 10 500 python $R/bench.py > $O/bench_n1.json 2> $O/bench_n1.err &&
for cfg in c4crc c3crc c3nest; do
  timeout -k 10 200 python $R/bench.py --config $cfg --no-cpu-baseline --no-extras --steps 10 --warmup 2 > $O/bench_$cfg.json 2> $O/bench_$cfg.err || exit $?
done &&
for cfg in c3 c4 c2 c3crc c4crc; do
  timeout -k 10 200 python $R/bench.py --op write --config $cfg --no-cpu-baseline --no-extras --steps 5 --warmup 2 > $O/write_$cfg.json 2> $O/write_$cfg.err || exit $?
done
