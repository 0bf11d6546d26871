mkdir -p gpurun_out/r03
timeout -k 10 100 ./tools/microbench/valu_bench > gpurun_out/r03/valu_bench.txt 2>&1 || exit 1
timeout -k 10 500 python3 -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r03/gpu_tests.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/r03/gpu_tests.log | head -20; tail -3 gpurun_out/r03/gpu_tests.log; exit 1; }
tail -1 gpurun_out/r03/gpu_tests.log
timeout -k 10 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r03/bench_head.json 2> gpurun_out/r03/bench_head.err || exit 1
timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-ttfs --steps 300 > gpurun_out/r03/bench_head_300.json 2>&1
