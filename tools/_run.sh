set -e
timeout -k 10 900 python3 -m pytest tests -x -q -m gpu > gpurun_out/gpu_all.log 2>&1
timeout -k 10 400 python3 tools/shard_cost.py > gpurun_out/shard_cost3.txt 2>&1
