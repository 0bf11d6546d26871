set -e
mkdir -p gpurun_out/r03/c5
timeout -k 10 300 python3 bench.py --workload c5 --samples-per-gpu 1048576 --steps 30 --warmup 20 --no-cpu-baseline --no-ttfs > gpurun_out/r03/c5/bench_c5_1M.json 2> gpurun_out/r03/c5/bench.err
tail -1 gpurun_out/r03/c5/bench_c5_1M.json | cut -c1-400
export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/r03/c5/fetch -o run --output-format csv -- python3 $R/bench.py --workload c5 --samples-per-gpu 1048576 --steps 30 --warmup 20 --no-cpu-baseline --no-ttfs > gpurun_out/r03/c5/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/r03/c5/write -o run --output-format csv -- python3 $R/bench.py --workload c5 --samples-per-gpu 1048576 --steps 30 --warmup 20 --no-cpu-baseline --no-ttfs > gpurun_out/r03/c5/write.log 2>&1
echo done
