#!/bin/bash
# Round 4: the index-CRC publish without __threadfence (current) vs the fenced one
# (libzarrhip_prevcrc.so, built from the previous commit's kernels): the bench's small read
# (one-shot 64^3 region, device-resident c4 shard) interleaved, then one kernel trace of each.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04m
mkdir -p "$OUT"
export TMPDIR=/tmp
OTHER=$R/zarr-java_amd/zarrhip/libzarrhip_prevcrc.so
cd "$R" || exit 1
for rep in 1 2 3; do
  for lib in cur prev; do
    if [ $lib = prev ]; then export ZH_LIB_PATH=$OTHER; else unset ZH_LIB_PATH; fi
    timeout -k 10 200 python3 profiles/small_read_trace.py 300 > "$OUT/${lib}_$rep.txt" 2> "$OUT/${lib}_$rep.err" || exit $?
    echo "$lib rep=$rep $(cat "$OUT/${lib}_$rep.txt")" >&2
  done
done
cd /tmp || exit 1
for lib in cur prev; do
  if [ $lib = prev ]; then export ZH_LIB_PATH=$OTHER; else unset ZH_LIB_PATH; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_$lib" -o run -- python3 "$R/profiles/small_read_trace.py" 100 > "$OUT/trace_$lib.txt" 2>&1 || exit $?
done
unset ZH_LIB_PATH
cd "$R" || exit 1
timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-host-inclusive > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
echo done >&2
