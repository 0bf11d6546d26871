mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/gpu_tests.log | head -20; tail -3 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
bash tools/ab.sh 3 300 prev=_ab/prev new=. || exit 1
for f in gpurun_out/ab/*.json; do python3 -c "import json;d=json.loads(open('$f').read().splitlines()[-1]);print('$f',d['roofline']['kernel_ms']['k_fold_r2'])"; done
