#!/bin/bash
# GPU step of the build -> measure loop: parity tests, A/B against _ab/prev, SQ counters of both.
mkdir -p gpurun_out/r03
timeout -k 10 500 python3 -u -m pytest tests -x -q -m gpu --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/r03/gpu_tests.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/r03/gpu_tests.log | head -20; tail -3 gpurun_out/r03/gpu_tests.log; exit 1; }
tail -1 gpurun_out/r03/gpu_tests.log
bash tools/ab_drv.sh 2 prev=_ab/prev new=. || exit 1
bash tools/pmc_sq.sh gpurun_out/r03/pmc_new || exit 1
(cd _ab/prev && GRAFT_REPO_ROOT=$PWD bash tools/pmc_sq.sh pmc_prev) || exit 1
mv _ab/prev/pmc_prev gpurun_out/r03/pmc_prev
python3 tools/pmc_summary.py gpurun_out/r03/pmc_new --skip 25 2>&1 | head -20
python3 tools/pmc_summary.py gpurun_out/r03/pmc_prev --skip 25 2>&1 | head -20
