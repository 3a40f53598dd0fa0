#!/bin/bash
set -o pipefail
# batches in flight 2 vs 3 at C1 / C3 / C4 / C5 (20 timed steps, 5 warmup), interleaved x2
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/inflc; cd $R
for rep in 1 2; do
  for c in c1 c3 c4 c5; do
    for v in 2 3; do
      timeout -k 10 150 python3 bench.py --config $c --steps 20 --warmup 5 --inflight $v --no-cpu-baseline --no-e2e --hbm-config '' > gpurun_out/inflc/r${rep}_${c}_$v.json 2> gpurun_out/inflc/r${rep}_${c}_$v.err || { tail -5 gpurun_out/inflc/r${rep}_${c}_$v.err; exit 1; }
      python3 -c "import json,sys; r=json.loads(open('gpurun_out/inflc/r${rep}_${c}_$v.json').read().strip().splitlines()[-1]); print('rep $rep $c inflight $v parse_cus %d ms_per_step %.4f value %.4g' % (r['config']['parse_cus'], r['ms_per_step'], r['value']))"
    done
  done
done
