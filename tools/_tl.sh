#!/bin/bash
# k_step phase timelines (tools/timeline.py) from a diagnostic build with stamps:
# the default build carries none (kgmt_kernels.hip, SBMP_TIMELINE).
set -e
rm -rf _ab/tl && mkdir -p _ab/tl
tar --exclude=./_ab --exclude=./.git --exclude=./gpurun_out --exclude='*/_obj' -cf - . | tar -xf - -C _ab/tl
(cd _ab/tl && SBMP_HIPCC_FLAGS=-DSBMP_TIMELINE python3 -m cudasbmp_amd.build --force > /dev/null)
mkdir -p gpurun_out/r03/tl_new
out=$PWD/gpurun_out/r03/tl_new
cd _ab/tl
SBMP_TIMELINE_ITER=20 SBMP_TIMELINE_OUT=$out/it20.bin timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-ttfs --steps 30 --warmup 20 > $out/b20.json 2>&1
SBMP_TIMELINE_ITER=1 SBMP_TIMELINE_OUT=$out/it1.bin timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-ttfs --steps 30 --warmup 20 > $out/b1.json 2>&1
