#!/bin/bash
# Round 4: file read/write and shim tests, the GPU suite and smoke (index-CRC publish without
# fences, zh_array_write_files), the index-CRC publish A/B on the small read, the bench line.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04n
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
step filetests 300 python3 -u -m pytest tests/test_gpu_files.py tests/test_jni_shim.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider
step gputests 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step smoke 200 python3 -c "import __graft_entry__ as g; g.smoke()"
OTHER=$R/zarr-java_amd/zarrhip/libzarrhip_prevcrc.so
for rep in 1 2 3; do
  for lib in cur prev; do
    if [ $lib = prev ]; then export ZH_LIB_PATH=$OTHER; else unset ZH_LIB_PATH; fi
    step sr_${lib}_$rep 200 python3 profiles/small_read_trace.py 300
    echo "$lib rep=$rep $(cat "$OUT/sr_${lib}_$rep.out")" >&2
  done
done
cd /tmp || exit 1
for lib in cur prev; do
  if [ $lib = prev ]; then export ZH_LIB_PATH=$OTHER; else unset ZH_LIB_PATH; fi
  step trace_$lib 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_$lib" -o run -- python3 "$R/profiles/small_read_trace.py" 100
done
unset ZH_LIB_PATH
cd "$R" || exit 1
step bench 600 python3 bench.py --steps 20 --warmup 5
echo done >&2
