#!/bin/bash
# A/B bench on one GPU box: tools/ab.sh <reps> <steps> <name>=<dir>[,VAR=value...] ...  (run from the repo root)
# Interleaves the variants rep by rep; prints G samples/s, us per step, the hot kernel's
# mean launch time (us) and its roofline fraction.  VAR=value pairs are set for that variant only.
reps=$1; steps=$2; shift 2
mkdir -p gpurun_out/ab
for rep in $(seq 1 $reps); do
  for spec in "$@"; do
    name=${spec%%=*}; rest=${spec#*=}
    dir=${rest%%,*}; envs=""
    [[ "$rest" == *,* ]] && envs=$(echo "${rest#*,}" | tr ',' ' ')
    out=$PWD/gpurun_out/ab/${name}_$rep.json
    (cd $dir && env $envs timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-ttfs --steps $steps > $out 2>/dev/null) || { echo "bench $name rc=$?"; exit 1; }
    python3 -c "import json;d=json.loads(open('$out').read().splitlines()[-1]);r=d['roofline'];print('$name',round(d['value']/1e9,3),round(d['ms_per_step']*1e3,2),r['avg_launch_us'],r['frac'])"
  done
done
