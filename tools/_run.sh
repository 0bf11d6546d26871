set -e
timeout -k 10 900 python3 -m pytest tests -x -q -m gpu > gpurun_out/gpu_step.log 2>&1
for i in 1 2; do timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-ttfs >> gpurun_out/b7.json 2>>gpurun_out/b7.err; done
SBMP_TIMELINE_ITER=45 SBMP_TIMELINE_OUT=gpurun_out/tls5.bin timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-ttfs > /dev/null 2>&1
