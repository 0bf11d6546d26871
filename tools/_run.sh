mkdir -p gpurun_out
timeout -k 10 300 python3 bench.py --workload c5 --no-ttfs --cpu-seconds 10 > gpurun_out/bench_c5_grid.json 2> gpurun_out/c5g.err || { echo "c5 grid rc=$?"; tail -5 gpurun_out/c5g.err; exit 1; }
tail -1 gpurun_out/bench_c5_grid.json | cut -c1-600
SBMP_EXPAND_VARIANT=5 timeout -k 10 300 python3 bench.py --workload c5 --no-ttfs --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/bench_c5_global.json 2> gpurun_out/c5l.err || { echo "c5 global rc=$?"; tail -5 gpurun_out/c5l.err; exit 1; }
tail -1 gpurun_out/bench_c5_global.json | cut -c1-600
SBMP_STEP=0 timeout -k 10 300 python3 bench.py --no-ttfs --no-cpu-baseline --steps 300 > gpurun_out/bench_c3_twolaunch.json 2> gpurun_out/c3t.err || { echo "c3 two-launch rc=$?"; exit 1; }
timeout -k 10 300 python3 bench.py --no-ttfs --no-cpu-baseline --steps 300 > gpurun_out/bench_c3_kstep300.json 2> gpurun_out/c3k.err || { echo "c3 rc=$?"; exit 1; }
for f in bench_c3_twolaunch bench_c3_kstep300; do python3 -c "import json;d=json.loads(open('gpurun_out/$f.json').read().splitlines()[-1]);print('$f',d['value']/1e9,d['roofline']['kernel_ms'])"; done
