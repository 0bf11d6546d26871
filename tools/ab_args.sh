#!/bin/bash
# A/B of any bench form: tools/ab_args.sh <reps> "<bench args>" name=dir ...  (run from the repo root on the GPU box)
# Prints G samples/s, us per step and the hot kernel's mean launch time per run, variants interleaved.
reps=$1; args=$2; shift 2
mkdir -p gpurun_out/ab
for rep in $(seq 1 $reps); do
  for spec in "$@"; do
    name=${spec%%=*}; dir=${spec#*=}
    out=$PWD/gpurun_out/ab/${name}_$rep.json
    (cd $dir && timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-ttfs $args > $out 2>/dev/null) || { echo "bench $name rc=$?"; exit 1; }
    python3 -c "import json;d=json.loads(open('$out').read().splitlines()[-1]);r=d['roofline'];print('$name',round(d['value']/1e9,3),round(d['ms_per_step']*1e3,2),r['avg_launch_us'])"
  done
done
