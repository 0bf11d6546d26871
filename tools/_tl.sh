mkdir -p gpurun_out/r03/tl
SBMP_TIMELINE_ITER=20 SBMP_TIMELINE_OUT=gpurun_out/r03/tl/it20.bin timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-ttfs --steps 30 --warmup 20 > gpurun_out/r03/tl/b20.json 2>&1 || exit 1
SBMP_TIMELINE_ITER=45 SBMP_TIMELINE_OUT=gpurun_out/r03/tl/it45.bin timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-ttfs --steps 30 --warmup 20 > gpurun_out/r03/tl/b45.json 2>&1 || exit 1
timeout -k 10 120 python3 tools/iter_times.py 60 > gpurun_out/r03/tl/iter_times.txt 2>&1
