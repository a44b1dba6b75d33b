#!/bin/bash
# Round 6 lab (DESIGN §4 "The chunk-CRC encode"): does the c4crc tile
# encode's 1.059x write traffic (split 32-B sectors of payloads at 4 mod 16) cost time?  The
# product library (non-temporal payload stores) against the lab build whose stores go through
# the cache (L2 merges the split sectors), alternated twice on one box: kernel time from the
# rocprofv3 kernel trace, WRITE_SIZE / FETCH_SIZE from separate PMC passes.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r06enc
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
cd /tmp || exit 1
W="python3 $R/bench.py --no-cpu-baseline --no-extras --no-host-inclusive --op write --config c4crc"
for pass in 1 2; do
  for lib in product lab; do
    if [ $lib = lab ]; then export ZH_LIB_PATH=$R/zarr-java_amd/zarrhip/libzarrhip_lab_enc_cached.so; else unset ZH_LIB_PATH; fi
    D="$OUT/${lib}_$pass"
    mkdir -p "$D"
    step wtrace_${lib}_$pass 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$D/wtrace_c4crc" -o run -- $W --steps 3 --warmup 1
    step wfetch_${lib}_$pass 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$D/wfetch_c4crc" -o run -- $W --steps 2 --warmup 1
    step wwrite_${lib}_$pass 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$D/wwrite_c4crc" -o run -- $W --steps 2 --warmup 1
    step wsum_${lib}_$pass 60 python3 $R/profiles/pmc_summary_write.py "$D" c4crc "$D/write_c4crc_summary.json" 206161575936
  done
done
unset ZH_LIB_PATH
echo done >&2
