#!/bin/bash
# PMC passes over a short bench run (run on the GPU box from the repo root):
#   tools/profile_pmc.sh <outdir> [extra bench.py arguments, e.g. --workload c5]
# Separate passes: SQ instruction/cycle counters, FETCH_SIZE, WRITE_SIZE
# (MI355X_MICROARCH.md: TCC slots cannot hold FETCH_SIZE and WRITE_SIZE together).
# Counters only with --pmc (no sys/runtime trace domains in the same run).
set -euo pipefail
OUT=${1:-gpurun_out/pmc}
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
mkdir -p "$R/$OUT"
ARGS="--steps 30 --warmup 20 --no-cpu-baseline --no-ttfs ${*:2}"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY -d "$R/$OUT/sq" -o run --output-format csv -- python3 "$R/bench.py" $ARGS > "$R/$OUT/sq.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT -d "$R/$OUT/sq2" -o run --output-format csv -- python3 "$R/bench.py" $ARGS > "$R/$OUT/sq2.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$R/$OUT/fetch" -o run --output-format csv -- python3 "$R/bench.py" $ARGS > "$R/$OUT/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$R/$OUT/write" -o run --output-format csv -- python3 "$R/bench.py" $ARGS > "$R/$OUT/write.log" 2>&1
