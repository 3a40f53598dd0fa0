#!/bin/bash
set -o pipefail
# E2E CLI at C3 and C5 with the native ingest's phase split (stderr), then
# single-batch kernel stats at C3/C4/C5
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out; cd $R
for c in c3 c5; do
  MPC_INGEST_TIMING=1 timeout -k 10 400 python -u bench.py --config $c --steps 5 --warmup 2 --kernel-reps 3 --no-cpu-baseline \
    --hbm-config "" > gpurun_out/e2e_$c.log 2> gpurun_out/e2e_$c.err || { tail -20 gpurun_out/e2e_$c.err; exit 1; }
  echo "== $c"; grep -o '"e2e": {[^}]*}[^}]*}' gpurun_out/e2e_$c.log; grep "^ingest" gpurun_out/e2e_$c.err | tail -24
done
bash scripts/kstats_configs.sh r04k c3 c4 c5
