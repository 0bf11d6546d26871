mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/gpu_tests.log | head -20; tail -3 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
bash tools/ab.sh 3 300 prev=_ab/prev new=. || exit 1
SBMP_TIMELINE_ITER=45 SBMP_TIMELINE_OUT=gpurun_out/tl_v.bin timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-ttfs > gpurun_out/b_tl_v.json 2>&1 || { echo "tl rc=$?"; exit 1; }
python3 tools/timeline.py gpurun_out/tl_v.bin --step | head -16
