#!/bin/bash
# Round 3: aligned decode tests + A/B, then the write-path PMC passes (run_r03_wpmc.sh).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash "$R/profiles/run_r03_align.sh" && bash "$R/profiles/run_r03_wpmc.sh"
