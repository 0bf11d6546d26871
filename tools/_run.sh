mkdir -p gpurun_out
timeout -k 10 300 python3 bench.py > gpurun_out/b_official.json 2> gpurun_out/b_official.err || { echo "bench rc=$?"; tail -5 gpurun_out/b_official.err; exit 1; }
tail -1 gpurun_out/b_official.json
bash tools/profile_round.sh gpurun_out/r01
