mkdir -p gpurun_out/r03
timeout -k 10 600 python3 -u -m pytest tests -x -v -m gpu -k "local_shard or rccl or two_processes or c4_local" --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/r03/gpu_sh.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/r03/gpu_sh.log | tail -25
exit $rc
