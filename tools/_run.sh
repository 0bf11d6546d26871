mkdir -p gpurun_out/r03
timeout -k 10 500 python3 -u -m pytest tests -x -q -m gpu --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/r03/gpu_tests.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/r03/gpu_tests.log | head -20; tail -3 gpurun_out/r03/gpu_tests.log; exit 1; }
tail -1 gpurun_out/r03/gpu_tests.log
bash tools/ab_drv.sh 2 prev=_ab/prev new=. || exit 1
timeout -k 10 120 python3 tools/iter_times.py 30 > gpurun_out/r03/iter_times_new.txt 2>&1 || exit 1
bash tools/_tl.sh || exit 1
