#!/bin/bash
# Full bench line (CPU port baseline, E2E where defined) + rocprofv3 kernel stats per config:
#   bash scripts/final_configs.sh <tag> c2 c1 ...   -> gpurun_out/<tag>_<config>_bench.json, <tag>_<config>/ (kernel stats)
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
cd $R && mkdir -p gpurun_out
for c in "$@"; do
  timeout -k 10 400 python3 -u bench.py --config $c > gpurun_out/${TAG}_$c.log 2>&1 || { echo "bench $c failed"; tail -5 gpurun_out/${TAG}_$c.log; exit 1; }
  grep '^{' gpurun_out/${TAG}_$c.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); json.dump(d, open('gpurun_out/${TAG}_${c}_bench.json','w'), indent=1); print('$c', '%.3e b/s' % d['value'], '%.1f us/step' % (1e3*d['ms_per_step']), 'parse %.1f us' % d['roofline']['mean_launch_us'], 'frac %.4f' % d['roofline']['frac'])"
done
bash $R/scripts/kstats_configs.sh $TAG "$@"
