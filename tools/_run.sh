mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/gpu_tests.log | head -20; tail -3 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
for rep in 1 2 3; do for v in wt new; do
  if [ $v = wt ]; then dir=_ab/wt; else dir=.; fi
  (cd $dir && timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-ttfs --steps 200 > /root/repo/gpurun_out/ab_${v}_$rep.json 2>/dev/null) || { echo "bench $v rc=$?"; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/ab_${v}_$rep.json').read().splitlines()[-1]);print('$v',d['value']/1e9,d['ms_per_step']*1e3,d['roofline']['avg_launch_us'])"
done; done
