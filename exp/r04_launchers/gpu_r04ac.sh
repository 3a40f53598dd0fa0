#!/bin/bash
set -o pipefail
# C2 batches in flight at the driver's step count (20 timed, 5 warmup), interleaved x3
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/infl20b; cd $R
for rep in 1 2 3; do
  for v in "3 176" "3 192" "3 208" "3 224" "4 160" "4 192"; do
    set -- $v
    timeout -k 10 120 python3 bench.py --config c2 --steps 20 --warmup 5 --inflight $1 --parse-cus $2 --no-cpu-baseline --no-e2e --hbm-config '' > gpurun_out/infl20b/r${rep}_$1_$2.json 2> gpurun_out/infl20b/r${rep}_$1_$2.err || { tail -5 gpurun_out/infl20b/r${rep}_$1_$2.err; exit 1; }
    python3 -c "import json,sys; r=json.loads(open('gpurun_out/infl20b/r${rep}_$1_$2.json').read().strip().splitlines()[-1]); print('rep $rep inflight $1 parse_cus $2 ms_per_step %.4f value %.4g' % (r['ms_per_step'], r['value']))"
  done
done
