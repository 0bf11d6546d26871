#!/bin/bash
# One SQ counter pass over a short bench run (GPU box, repo root):  tools/pmc_sq.sh <outdir> [bench args]
# Per-wave instruction counts of the hot kernel: python3 tools/pmc_summary.py <outdir> --skip 25
set -euo pipefail
OUT=${1:-gpurun_out/pmc_sq}
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
mkdir -p "$R/$OUT"
ARGS="--steps 30 --warmup 20 --no-cpu-baseline --no-ttfs ${*:2}"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY -d "$R/$OUT/sq" -o run --output-format csv -- python3 "$R/bench.py" $ARGS > "$R/$OUT/sq.log" 2>&1
