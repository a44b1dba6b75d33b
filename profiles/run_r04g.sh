#!/bin/bash
# Round 4: the PCIe ceiling for the host-terminated read (page-locked copies of 128 MiB slabs,
# each direction alone and both at once), then the default bench line on the same box.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04g
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
step pcie 300 python3 profiles/pcie_lab.py 64 3
step bench 500 python3 bench.py --steps 20 --warmup 5
echo done >&2
