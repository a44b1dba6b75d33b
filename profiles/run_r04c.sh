#!/bin/bash
# Round 4: the JNI critical-window lab (2 GiB sub-shard read through arrayReadPieces per
# ZH_JNI_SLAB_MB cap), then the headline c4 decode's kernel trace and FETCH/WRITE passes with the
# current binary (profiles/r04/c4_summary.json), and the 2-rank strong-mode rehearsal of the
# driver's multi-GPU command (both ranks on the one card: gloo stands in for RCCL).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04c
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  echo "== $name: $*" >&2
  timeout -k 10 "$t" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  echo "== $name rc=$rc" >&2
  if [ $rc -ne 0 ]; then tail -n 40 "$OUT/$name.out" "$OUT/$name.err" >&2; exit $rc; fi
}
cd "$R" || exit 1
step jnilab 400 python3 -u profiles/jni_window_lab.py "$OUT/jni_window_lab.json"
cd /tmp || exit 1
B="python3 $R/bench.py --no-cpu-baseline --no-extras --no-host-inclusive"
for cfg in c4; do
  step trace_$cfg 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_$cfg" -o run -- $B --config $cfg --steps 5 --warmup 2
  step pmc_fetch_$cfg 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch_$cfg" -o run -- $B --config $cfg --steps 2 --warmup 1
  step pmc_write_$cfg 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write_$cfg" -o run -- $B --config $cfg --steps 2 --warmup 1
  step sum_$cfg 60 python3 $R/profiles/pmc_summary.py "$OUT" $cfg "$OUT/${cfg}_summary.json"
done
cd "$R" || exit 1
step strong2 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --no-host-out
echo done >&2
