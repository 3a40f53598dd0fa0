#!/bin/bash
set -o pipefail
# Round-4 final measurements, part 2: the bench line of every other config and
# single-batch kernel stats of all five
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for c in c1 c3 c4 c5; do
  timeout -k 10 400 python3 -u bench.py --config $c > gpurun_out/f4_$c.log 2>&1 || { echo "bench $c failed"; tail -5 gpurun_out/f4_$c.log; exit 1; }
  grep '^{' gpurun_out/f4_$c.log | tail -1 > gpurun_out/f4_${c}_bench.json
  python3 -c "import json; d=json.load(open('gpurun_out/f4_${c}_bench.json')); print('$c', '%.3e' % d['value'], '%.1f us/step' % (1e3*d['ms_per_step']), 'single %.1f' % (1e3*(d.get('single_batch_ms_per_step') or 0)), 'e2e', (d.get('e2e') or {}).get('wall_s'))"
done
bash scripts/kstats_configs.sh f4k c1 c2 c3 c4 c5 || exit 1
