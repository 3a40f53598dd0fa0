#!/bin/bash
set -o pipefail
# final bench line of every config with the final kernels and the per-config
# in-flight defaults (C1 4, C2 3, C3-C5 2)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for c in c1 c3 c4 c5; do
  timeout -k 10 400 python3 -u bench.py --config $c --hbm-config '' > gpurun_out/f4g_$c.log 2>&1 || { echo "bench $c failed"; tail -5 gpurun_out/f4g_$c.log; exit 1; }
  grep '^{' gpurun_out/f4g_$c.log | tail -1 > gpurun_out/f4g_${c}_bench.json
  python3 -c "
import json; r=json.load(open('gpurun_out/f4g_${c}_bench.json'))
print('$c', 'value %.4g' % r['value'], 'us/step %.1f' % (r['ms_per_step']*1e3), 'single %.1f' % (r['single_batch_ms_per_step']*1e3), 'inflight', r['config']['batches_in_flight'], 'kparse %.1f' % r['roofline']['mean_launch_us'], 'e2e %.3f' % (r['e2e']['wall_s'] if r.get('e2e') else -1))"
done
