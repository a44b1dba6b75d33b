#!/bin/bash
# Round 3 (session 2): GPU tests, then the aligned tile-encode A/B (ZH_ENC_ALIGN), then the
# default bench line with the current binary.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03e
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  echo "== $name: $*" >&2
  timeout -k 10 "$t" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  echo "== $name rc=$rc" >&2
  if [ $rc -ne 0 ]; then exit $rc; fi
}
cd "$R" || exit 1
step pytest 900 python3 -u -m pytest tests -m gpu -x -v --timeout 170 --timeout-method thread
step smoke 120 python3 -c "import __graft_entry__ as g; g.smoke()"
cd /tmp || exit 1
step ab_enc_aln 400 python3 $R/profiles/ab_write_env.py c4crc 2 4 - ZH_ENC_ALIGN=1 ZH_ENC_ALIGN=1,ZH_ENC_ALIGN_PF=0
step bench 600 python3 $R/bench.py
