mkdir -p gpurun_out/r03
timeout -k 10 60 ./tools/microbench/salu_bench > gpurun_out/r03/salu_bench.txt 2>&1 || true
timeout -k 10 500 python3 -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r03/gpu_tests.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/r03/gpu_tests.log | head -20; tail -3 gpurun_out/r03/gpu_tests.log; exit 1; }
tail -1 gpurun_out/r03/gpu_tests.log
bash tools/ab_drv.sh 3 prev=_ab/prev new=. || exit 1
bash tools/pmc_sq.sh gpurun_out/r03/pmc_new || exit 1
