#!/bin/bash
# round 6: parse CUs / batches in flight at C2 and C1 with the current kernels (bench lines only)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/sweep
run() {  # cfg inflight parse_cus
  timeout -k 10 180 python3 -u bench.py --config $1 --inflight $2 --parse-cus $3 --no-cpu-baseline --no-e2e --hbm-config none \
    --kernel-reps 3 > gpurun_out/sweep/$1_$2_$3.json 2> gpurun_out/sweep/$1_$2_$3.err || { echo "fail $1 $2 $3"; tail -5 gpurun_out/sweep/$1_$2_$3.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], '%.4g' % d['value'], '%.1f us/step' % (1000*d['ms_per_step']))" gpurun_out/sweep/$1_$2_$3.json "$1 inflight $2 parse_cus $3"
}
for pc in 192 176 208 224 160 192; do run c2 3 $pc; done
run c2 4 192
run c2 4 208
for pc in 96 80 112 128; do run c1 4 $pc; done
