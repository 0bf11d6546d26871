#!/bin/bash
# Kernel-trace a short bench run (GPU box, repo root):  tools/trace_bench.sh <outdir> [bench args...]
# Writes <outdir>/bench.json (the bench line) and <outdir>/trace/run_kernel_{trace,stats}.csv.
set -euo pipefail
OUT=${1:-gpurun_out/trace}; shift || true
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
mkdir -p "$R/$OUT"
ARGS="${*:---no-cpu-baseline --no-ttfs}"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/$OUT/trace" -o run --output-format csv -- python3 "$R/bench.py" $ARGS > "$R/$OUT/bench.json" 2> "$R/$OUT/bench.err"
