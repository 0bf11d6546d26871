set -e
mkdir -p gpurun_out/r03/c5ab
timeout -k 10 500 python3 -u -m pytest tests -x -q -m gpu --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/r03/gpu_tests.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/r03/gpu_tests.log | head; exit 1; }
tail -1 gpurun_out/r03/gpu_tests.log
for rep in 1 2; do for v in prev new; do
  d=.; [ $v = prev ] && d=_ab/prev
  (cd $d && timeout -k 10 200 python3 bench.py --workload c5 --samples-per-gpu 1048576 --steps 30 --warmup 20 --no-cpu-baseline --no-ttfs) > gpurun_out/r03/c5ab/${v}_$rep.json 2>/dev/null
  python3 -c "import json;d=json.loads(open('gpurun_out/r03/c5ab/${v}_$rep.json').read().strip().splitlines()[-1]);r=d['roofline'];print('$v',round(d['value']/1e9,3),r['avg_launch_us'],r['kernel_ms'])"
done; done
export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/r03/c5ab/fetch -o run --output-format csv -- python3 $R/bench.py --workload c5 --samples-per-gpu 1048576 --steps 30 --warmup 20 --no-cpu-baseline --no-ttfs > gpurun_out/r03/c5ab/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/r03/c5ab/write -o run --output-format csv -- python3 $R/bench.py --workload c5 --samples-per-gpu 1048576 --steps 30 --warmup 20 --no-cpu-baseline --no-ttfs > gpurun_out/r03/c5ab/write.log 2>&1
echo done
