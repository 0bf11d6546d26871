#!/bin/bash
# The GPU side of the build -> measure loop (run on the GPU box from the repo root, through
# gpurun).  Every step runs under its own time limit; the first failing step ends the call.
#
#   tools/gpu_cycle.sh tests <out>                 pytest -m gpu (log in <out>/gpu_tests.log)
#   tools/gpu_cycle.sh tests_k <out> <expr>        the -m gpu tests matching -k <expr>
#   tools/gpu_cycle.sh ab <out> <reps> name=dir..  A/B of the driver's bench form (20 after 5)
#                                                  and a 300-step line, runs interleaved
#   tools/gpu_cycle.sh abenv <out> <reps> name=VAR=v..  the same A/B in this tree, each side with one
#                                                  environment setting (e.g. off=SBMP_OVERLAP=0 on=SBMP_OVERLAP=1)
#   tools/gpu_cycle.sh timeline <out> <dir> <it>.. k_step phase stamps at iterations <it> from the
#                                                  stamped build in <dir> (tools/mk_variant.sh tl)
#   tools/gpu_cycle.sh sq <out> [bench args]       one SQ counter pass (tools/pmc_summary.py)
#   tools/gpu_cycle.sh pmc <out> [bench args]      SQ, SQ2, FETCH_SIZE, WRITE_SIZE passes
#   tools/gpu_cycle.sh trace <out> [bench args]    rocprofv3 --kernel-trace --stats of a bench run
#   tools/gpu_cycle.sh bench <out> <name> [args]   one bench line into <out>/<name>.json
#   tools/gpu_cycle.sh shard <out>                 tools/shard_cost.py 1 2 8 and two ranks on one GPU
#   tools/gpu_cycle.sh attrib <out> <wl> <n> <it>  per-launch traffic fitted per child (tools/write_attrib.py)
#   tools/gpu_cycle.sh wlpmc <out> <wl> <n> <N> <first> <last>  SQ / FETCH / WRITE of k_step summed over
#                                                  iterations first..last of one seeded run (tools/pmc_workload.py)
#   tools/gpu_cycle.sh microbench <out>            build and run tools/microbench/{valu,salu}_bench
#   tools/gpu_cycle.sh final <out>                 the round's record: pytest -m gpu, the default bench line,
#                                                  two driver-form lines, a 300-step line, the rocprofv3
#                                                  kernel-trace summary of the default line, c5 at 131,072
#
# Several steps in one call:  tools/gpu_cycle.sh tests o && tools/gpu_cycle.sh ab o 2 prev=_ab/prev new=.
set -uo pipefail
cmd=$1; out=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/$out"
line() {   # value (G samples/s), ms per step, k_step us of a bench JSON line
    python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d['roofline'];print(sys.argv[2],round(d['value']/1e9,3),round(d['ms_per_step']*1e3,2),r.get('avg_launch_us'),r.get('frac'))" "$1" "$2"
}
case $cmd in
tests)
    timeout -k 10 600 python3 -u -m pytest tests -x -q -m gpu --timeout 180 --timeout-method thread \
        -p no:cacheprovider > "$R/$out/gpu_tests.log" 2>&1
    rc=$?; tail -2 "$R/$out/gpu_tests.log"
    [ $rc -eq 0 ] || { grep -E "FAILED|Error" "$R/$out/gpu_tests.log" | head -20; exit $rc; } ;;
tests_k)
    timeout -k 10 600 python3 -u -m pytest tests -x -v -m gpu -k "$1" --timeout 180 --timeout-method thread \
        -p no:cacheprovider > "$R/$out/gpu_tests_k.log" 2>&1
    rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" "$R/$out/gpu_tests_k.log" | tail -30; exit $rc ;;
ab)
    reps=$1; shift
    for rep in $(seq 1 "$reps"); do
        for spec in "$@"; do
            name=${spec%%=*}; dir=${spec#*=}
            for cfg in 20:5 300:20; do
                k=${cfg%%:*}; w=${cfg#*:}; f="$R/$out/${name}_${k}_$rep.json"
                (cd "$dir" && timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-ttfs --steps "$k" --warmup "$w" \
                    > "$f" 2> "$f.err") || { echo "bench $name rc=$?"; tail -5 "$f.err"; exit 1; }
                line "$f" "$name K=$k"
            done
        done
    done ;;
abenv)
    reps=$1; shift
    for rep in $(seq 1 "$reps"); do
        for spec in "$@"; do
            name=${spec%%=*}; kv=${spec#*=}
            for cfg in 20:5 300:20; do
                k=${cfg%%:*}; w=${cfg#*:}; f="$R/$out/${name}_${k}_$rep.json"
                env "$kv" timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-ttfs --steps "$k" --warmup "$w" \
                    > "$f" 2> "$f.err" || { echo "bench $name rc=$?"; tail -5 "$f.err"; exit 1; }
                line "$f" "$name K=$k"
            done
        done
    done ;;
timeline)
    dir=$1; shift
    for it in "$@"; do
        (cd "$dir" && SBMP_TIMELINE_ITER=$it SBMP_TIMELINE_OUT="$R/$out/it$it.bin" timeout -k 10 120 python3 bench.py \
            --no-cpu-baseline --no-ttfs --steps 30 --warmup 20 > "$R/$out/b$it.json" 2> "$R/$out/b$it.err") || exit 1
        python3 tools/timeline.py "$R/$out/it$it.bin" --step > "$R/$out/k_step_iter$it.txt" && head -30 "$R/$out/k_step_iter$it.txt"
    done ;;
sq)
    cd /tmp && export TMPDIR=/tmp
    timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES \
        SQ_BUSY_CYCLES SQ_WAIT_INST_ANY -d "$R/$out/sq" -o run --output-format csv -- python3 "$R/bench.py" \
        --steps 30 --warmup 20 --no-cpu-baseline --no-ttfs "$@" > "$R/$out/sq.log" 2>&1 || exit 1
    cd "$R" && python3 tools/pmc_summary.py "$out" --skip 25 > "$R/$out/sq_summary.txt" && sed -n 1,30p "$R/$out/sq_summary.txt" ;;
pmc)
    bash tools/profile_pmc.sh "$out" "$@" || exit 1
    python3 tools/pmc_summary.py "$out" --skip 25 > "$R/$out/pmc_summary.txt" && sed -n 1,40p "$R/$out/pmc_summary.txt" ;;
trace)
    cd /tmp && export TMPDIR=/tmp
    timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/$out/trace" -o run --output-format csv -- \
        python3 "$R/bench.py" "$@" > "$R/$out/bench.json" 2> "$R/$out/bench.err" || exit 1
    cd "$R" && line "$out/bench.json" traced ;;
bench)
    name=$1; shift
    timeout -k 10 300 python3 bench.py "$@" > "$R/$out/$name.json" 2> "$R/$out/$name.err" || { tail -5 "$R/$out/$name.err"; exit 1; }
    line "$R/$out/$name.json" "$name" ;;
shard)
    timeout -k 10 300 python3 tools/shard_cost.py 1 2 8 > "$R/$out/shard_cost.txt" 2>&1 || exit 1
    cat "$R/$out/shard_cost.txt"
    timeout -k 10 300 python3 bench.py --gpus 2 --collectives host --steps 50 --warmup 10 --no-cpu-baseline --no-ttfs \
        > "$R/$out/bench_2rank_host.json" 2> "$R/$out/bench_2rank_host.err" || { tail -5 "$R/$out/bench_2rank_host.err"; exit 1; }
    tail -1 "$R/$out/bench_2rank_host.json" ;;
final)
    timeout -k 10 900 python3 -u -m pytest tests -x -q -m gpu --timeout 180 --timeout-method thread \
        -p no:cacheprovider > "$R/$out/gpu_tests.log" 2>&1 || { tail -20 "$R/$out/gpu_tests.log"; exit 1; }
    tail -1 "$R/$out/gpu_tests.log"
    timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke()" > "$R/$out/smoke.log" 2>&1 \
        || { tail -5 "$R/$out/smoke.log"; exit 1; }
    tail -1 "$R/$out/smoke.log"
    timeout -k 10 300 python3 bench.py > "$R/$out/bench.json" 2> "$R/$out/bench.err" || { tail -5 "$R/$out/bench.err"; exit 1; }
    line "$R/$out/bench.json" default
    for rep in 1 2; do
        timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-ttfs > "$R/$out/drv_$rep.json" \
            2> "$R/$out/drv_$rep.err" || exit 1
        line "$R/$out/drv_$rep.json" "driver $rep"
    done
    timeout -k 10 200 python3 bench.py --steps 300 --warmup 20 --no-cpu-baseline --no-ttfs > "$R/$out/s300.json" \
        2> "$R/$out/s300.err" || exit 1
    line "$R/$out/s300.json" s300
    timeout -k 10 300 python3 bench.py --workload c5 --samples-per-gpu 131072 --warmup 5 --steps 35 --no-cpu-baseline --no-ttfs \
        > "$R/$out/c5_131k.json" 2> "$R/$out/c5_131k.err" || exit 1
    line "$R/$out/c5_131k.json" c5_131k
    cd /tmp && export TMPDIR=/tmp
    timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/$out/trace" -o run --output-format csv -- \
        python3 "$R/bench.py" --no-cpu-baseline > "$R/$out/bench_traced.json" 2> "$R/$out/bench_traced.err" || exit 1
    cd "$R" && line "$out/bench_traced.json" traced ;;
attrib)   # <workload> <samples> <iterations>: per-launch WRITE_SIZE / FETCH_SIZE fitted per unit of work
    wl=$1; ns=$2; it=$3; mkdir -p "$R/$out/$wl"; cd /tmp && export TMPDIR=/tmp
    for c in WRITE_SIZE FETCH_SIZE; do
        d=$(echo "$c" | cut -d_ -f1 | tr A-Z a-z)
        timeout -s KILL 120 rocprofv3 --pmc "$c" -d "$R/$out/$wl/$d" -o run --output-format csv -- \
            python3 "$R/tools/write_attrib.py" run "$wl" "$ns" "$it" "$R/$out/$wl/log.json" \
            > "$R/$out/$wl/$d.log" 2>&1 || { tail -5 "$R/$out/$wl/$d.log"; exit 1; }
    done
    cd "$R" && python3 tools/write_attrib.py fit "$out/$wl/log.json" "$out/$wl/write" "$out/$wl/fetch" \
        > "$out/$wl/fit.txt" && head -8 "$out/$wl/fit.txt" ;;
wlpmc)   # <workload> <samples> <iterations> <first> <last>
    wl=$1; ns=$2; it=$3; f0=$4; f1=$5; cd /tmp && export TMPDIR=/tmp
    for g in sq fetch write; do
        case $g in sq) ctr="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES";;
                   fetch) ctr=FETCH_SIZE;; write) ctr=WRITE_SIZE;; esac
        timeout -s KILL 120 rocprofv3 --pmc $ctr -d "$R/$out/$g" -o run --output-format csv -- \
            python3 "$R/tools/pmc_workload.py" run "$wl" "$ns" "$it" "$R/$out/log.json" \
            > "$R/$out/$g.log" 2>&1 || { tail -5 "$R/$out/$g.log"; exit 1; }
    done
    cd "$R" && python3 tools/pmc_workload.py sum "$out" "$f0" "$f1" --json "$out/pmc_${wl}_${ns}.json" \
        > "$out/summary.txt" && cat "$out/summary.txt" ;;
microbench)
    for b in valu_bench salu_bench; do
        /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 "tools/microbench/$b.hip" -o "/tmp/$b" || exit 1
        timeout -k 10 120 "/tmp/$b" > "$R/$out/$b.txt" || exit 1
        cat "$R/$out/$b.txt"
    done ;;
*)
    echo "unknown step $cmd"; exit 2 ;;
esac
