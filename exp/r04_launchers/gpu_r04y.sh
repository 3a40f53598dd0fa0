#!/bin/bash
set -o pipefail
# C1 batches in flight x parse-grid CUs (20 timed steps, 5 warmup), interleaved x3
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/inflc1; cd $R
for rep in 1 2 3; do
  for v in "2 128" "3 96" "3 128" "3 160" "4 96" "4 128"; do
    set -- $v
    timeout -k 10 100 python3 bench.py --config c1 --steps 20 --warmup 5 --inflight $1 --parse-cus $2 --no-cpu-baseline --no-e2e --hbm-config '' > gpurun_out/inflc1/r${rep}_$1_$2.json 2> gpurun_out/inflc1/r${rep}_$1_$2.err || { tail -5 gpurun_out/inflc1/r${rep}_$1_$2.err; exit 1; }
    python3 -c "import json,sys; r=json.loads(open('gpurun_out/inflc1/r${rep}_$1_$2.json').read().strip().splitlines()[-1]); print('rep $rep c1 inflight $1 parse_cus $2 ms_per_step %.4f value %.4g' % (r['ms_per_step'], r['value']))"
  done
done
