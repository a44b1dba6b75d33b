#!/bin/bash
# Round 6 closing run (one, on the final tree): the GPU suite as the driver
# runs it, smoke, the default bench line, the c4 kernel trace and its FETCH_SIZE / WRITE_SIZE
# passes (→ c4_summary.json), then one 2-rank strong-mode pass of bench.py on this one GPU to
# check the changed N > 1 code path (not scaling evidence: the ranks share the GPU).
# Records → gpurun_out/r06final.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r06final
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  echo "== $name: $*" >&2
  timeout -k 10 "$t" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  echo "== $name rc=$rc" >&2
  if [ $rc -ne 0 ]; then tail -n 60 "$OUT/$name.out" "$OUT/$name.err" >&2; exit $rc; fi
}
cd "$R" || exit 1
step gputests 800 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step smoke 200 python3 -c "import __graft_entry__ as g; g.smoke()"
step bench 500 python3 bench.py
cd /tmp || exit 1
B="python3 $R/bench.py --no-cpu-baseline --no-extras --no-host-inclusive --allocations 1 --config c4"
step trace_c4 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_c4" -o run -- $B --steps 5 --warmup 2
step pmc_fetch_c4 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch_c4" -o run -- $B --steps 2 --warmup 1
step pmc_write_c4 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write_c4" -o run -- $B --steps 2 --warmup 1
step sum_c4 60 python3 $R/profiles/pmc_summary.py "$OUT" c4 "$OUT/c4_summary.json"
cd "$R" || exit 1
step strong2 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --no-host-out
echo done >&2
