mkdir -p gpurun_out
for rep in 1 2 3; do for v in base head; do
  if [ $v = base ]; then dir=_ab/base; else dir=.; fi
  (cd $dir && timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-ttfs --steps 200 > /root/repo/gpurun_out/ab_${v}_$rep.json 2>/dev/null) || { echo "bench $v rc=$?"; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/ab_${v}_$rep.json').read().splitlines()[-1]);print('$v',d['value']/1e9,d['ms_per_step']*1e3,d['roofline']['achieved'])"
done; done
