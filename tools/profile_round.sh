#!/bin/bash
# Round profile (GPU box, repo root):  tools/profile_round.sh <outdir>
#   1. rocprofv3 --kernel-trace --stats of the default bench command
#   2. the PMC passes of tools/profile_pmc.sh (separate runs, counters only)
# Summaries are copied into profiles/ afterwards (tools/summarize_round.py).
set -euo pipefail
OUT=${1:-gpurun_out/round}
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/$OUT/trace" -o run --output-format csv \
    -- python3 "$R/bench.py" > "$R/$OUT/bench.json" 2> "$R/$OUT/bench.err"
cd "$R"
tools/profile_pmc.sh "$OUT/pmc"
