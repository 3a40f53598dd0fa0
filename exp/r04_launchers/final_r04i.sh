#!/bin/bash
set -o pipefail
# C5 and C2 bench lines after the K_left change for 512-thread plans
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for c in c5 c2; do
  timeout -k 10 400 python3 -u bench.py --config $c $( [ $c = c5 ] && echo --hbm-config= ) > gpurun_out/f4i_$c.log 2>&1 || { echo "bench $c failed"; tail -5 gpurun_out/f4i_$c.log; exit 1; }
  grep '^{' gpurun_out/f4i_$c.log | tail -1 > gpurun_out/f4i_${c}_bench.json
  python3 -c "
import json; r=json.load(open('gpurun_out/f4i_${c}_bench.json'))
print('$c', 'value %.4g' % r['value'], 'us/step %.1f' % (r['ms_per_step']*1e3), 'single %.1f' % (r['single_batch_ms_per_step']*1e3), 'e2e %.3f' % (r['e2e']['wall_s'] if r.get('e2e') else -1))"
done
