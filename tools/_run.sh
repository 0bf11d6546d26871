mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/gpu_tests.log | head -20; tail -3 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
