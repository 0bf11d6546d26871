mkdir -p gpurun_out/r03/tl_new
SBMP_TIMELINE_ITER=20 SBMP_TIMELINE_OUT=gpurun_out/r03/tl_new/it20.bin timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-ttfs --steps 30 --warmup 20 > gpurun_out/r03/tl_new/b20.json 2>&1 || exit 1
SBMP_TIMELINE_ITER=1 SBMP_TIMELINE_OUT=gpurun_out/r03/tl_new/it1.bin timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-ttfs --steps 30 --warmup 20 > gpurun_out/r03/tl_new/b1.json 2>&1 || exit 1
