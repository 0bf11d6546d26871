#!/bin/bash
# A/B of the driver form and a 300-step run, printing the fold's per-launch time:
#   tools/ab_fold.sh <reps> <name>=<dir> ...
reps=$1; shift
mkdir -p gpurun_out/ab
for rep in $(seq 1 $reps); do
  for spec in "$@"; do
    name=${spec%%=*}; dir=${spec#*=}
    for cfg in 20:5 300:20; do
      k=${cfg%%:*}; w=${cfg#*:}
      out=$PWD/gpurun_out/ab/${name}_${k}_$rep.json
      (cd $dir && timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-ttfs --steps $k --warmup $w > $out 2>/dev/null) || { echo "bench $name rc=$?"; exit 1; }
      python3 -c "import json;d=json.loads(open('$out').read().splitlines()[-1]);r=d['roofline'];f=r['kernel_ms'].get('k_fold_r2',{});print('$name K=$k',round(d['value']/1e9,3),round(d['ms_per_step']*1e3,2),r['avg_launch_us'],'fold',f.get('launches'),f.get('avg_us'))"
    done
  done
done
