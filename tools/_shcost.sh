mkdir -p gpurun_out/r03
timeout -k 10 300 python3 tools/shard_cost.py 1 2 8 > gpurun_out/r03/shard_cost.txt 2>&1 || exit 1
cat gpurun_out/r03/shard_cost.txt
timeout -k 10 300 python3 bench.py --gpus 2 --collectives host --steps 50 --warmup 10 --no-cpu-baseline --no-ttfs > gpurun_out/r03/bench_2rank_host.json 2> gpurun_out/r03/bench_2rank_host.err || { tail -5 gpurun_out/r03/bench_2rank_host.err; exit 1; }
tail -1 gpurun_out/r03/bench_2rank_host.json
