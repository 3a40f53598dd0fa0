#!/bin/bash
set -o pipefail
# after the K_left change for 512-thread plans: smoke, the GPU suite, the C5 and C2 bench lines
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/f4h_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/f4h_smoke.log; exit 1; }
tail -1 gpurun_out/f4h_smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/f4h_t.log 2>&1
rc=$?; grep -E "passed|failed|error" gpurun_out/f4h_t.log | tail -2; [ $rc -eq 0 ] || { grep -E "FAILED|^E " gpurun_out/f4h_t.log | head -30; exit $rc; }
for c in c5 c2; do
  timeout -k 10 400 python3 -u bench.py --config $c $( [ $c = c5 ] && echo --hbm-config= ) > gpurun_out/f4h_$c.log 2>&1 || { echo "bench $c failed"; tail -5 gpurun_out/f4h_$c.log; exit 1; }
  grep '^{' gpurun_out/f4h_$c.log | tail -1 > gpurun_out/f4h_${c}_bench.json
  python3 -c "
import json; r=json.load(open('gpurun_out/f4h_${c}_bench.json'))
print('$c', 'value %.4g' % r['value'], 'us/step %.1f' % (r['ms_per_step']*1e3), 'single %.1f' % (r['single_batch_ms_per_step']*1e3), 'e2e %.3f' % (r['e2e']['wall_s'] if r.get('e2e') else -1))"
done
