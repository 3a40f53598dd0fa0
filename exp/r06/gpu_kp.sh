#!/bin/bash
# round 6: parse-phase timings only (timing-only builds need not be exact)
#   bash exp/r06/gpu_kp.sh "<cfgs>" exp/v/a.so exp/v/b.so ...
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/kp
CFGS=$1; shift
for c in $CFGS; do
  KEXP_CFG=$c timeout -k 10 300 python3 -u scripts/kp_multi.py "$@" > gpurun_out/kp/kp_$c.log 2>&1 || { echo "kp $c failed"; tail -5 gpurun_out/kp/kp_$c.log; exit 1; }
  grep " us " gpurun_out/kp/kp_$c.log
done
