mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
grep -E "passed|failed|FAILED" gpurun_out/gpu_tests.log | tail -20
for rep in 1 2; do for w in 0 3 7 1; do
  SBMP_WT=$w timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-ttfs > gpurun_out/b_w${w}_$rep.json 2> gpurun_out/b_w${w}_$rep.err || { echo "bench $w rc=$?"; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/b_w${w}_$rep.json').read().splitlines()[-1]);print('wt',$w,d['value']/1e9,d['ms_per_step']*1e3,d['roofline']['achieved'])"
done; done
