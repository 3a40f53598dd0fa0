#!/bin/bash
set -o pipefail
# parse-grid CUs with 2 batches in flight at C3 / C4 / C5 with the final kernels (20 timed steps, 2 reps)
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/cus345; cd $R
for rep in 1 2; do
  for v in "c5 176" "c5 192" "c5 208" "c5 224" "c3 208" "c3 224" "c3 240" "c4 208" "c4 224" "c4 240"; do
    set -- $v
    timeout -k 10 150 python3 bench.py --config $1 --steps 20 --warmup 5 --parse-cus $2 --no-cpu-baseline --no-e2e --hbm-config= > gpurun_out/cus345/r${rep}_$1_$2.json 2> gpurun_out/cus345/r${rep}_$1_$2.err || { tail -5 gpurun_out/cus345/r${rep}_$1_$2.err; exit 1; }
    python3 -c "import json; r=json.loads(open('gpurun_out/cus345/r${rep}_$1_$2.json').read().strip().splitlines()[-1]); print('rep $rep $1 parse_cus $2 us_per_step %.1f' % (r['ms_per_step'] * 1e3))"
  done
done
