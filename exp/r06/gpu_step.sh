#!/bin/bash
# round 6: full single-batch steps of library variants (scripts/step_multi.py), timing only
#   bash exp/r06/gpu_step.sh "<cfgs>" exp/v/a.so exp/v/b.so ...
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/step
CFGS=$1; shift
for c in $CFGS; do
  KEXP_CFG=$c timeout -k 10 300 python3 -u scripts/step_multi.py "$@" > gpurun_out/step/step_$c.log 2>&1 || { echo "step $c failed"; tail -5 gpurun_out/step/step_$c.log; exit 1; }
  grep " us " gpurun_out/step/step_$c.log
done
