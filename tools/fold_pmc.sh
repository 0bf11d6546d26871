set -o pipefail
O=gpurun_out/r05/fold
mkdir -p $O
rocprofv3 -L > $O/avail.txt 2>&1 || true
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAIT_ANY -d $O/p1 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-ttfs --steps 20 --warmup 5 > $O/p1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD -d $O/p2 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-ttfs --steps 20 --warmup 5 > $O/p2.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/tr -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-ttfs --steps 20 --warmup 5 > $O/tr.log 2>&1
