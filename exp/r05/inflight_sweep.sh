#!/bin/bash
# batches in flight x parse CUs sweep for one config (20-step runs as the driver makes them, 2 interleaved reps)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
CFG=$1; shift
for rep in 1 2; do
for combo in "$@"; do
  IF=${combo%/*}; CU=${combo#*/}
  timeout -k 10 300 python3 -u bench.py --config $CFG --inflight $IF --parse-cus $CU --no-cpu-baseline --no-e2e --hbm-config "" > gpurun_out/sw_${CFG}_${IF}_${CU}.log 2>&1 || { echo "bench $combo failed"; tail -5 gpurun_out/sw_${CFG}_${IF}_${CU}.log; exit 1; }
  python3 -c "
import json,sys; d=json.loads([l for l in open('gpurun_out/sw_${CFG}_${IF}_${CU}.log') if l.startswith('{')][-1])
print('$CFG rep$rep inflight $IF cus $CU: %.1f us/step %.3e b/s timed-parse %.1f us' % (1e3*d['ms_per_step'], d['value'], (d.get('roofline_timed') or {}).get('mean_launch_us', 0)))"
done
done
