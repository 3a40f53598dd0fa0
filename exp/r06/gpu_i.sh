#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/r6i
for c in c3 c2; do
  KEXP_CFG=$c timeout -k 10 300 python3 -u scripts/kp_multi.py exp/v/nospec.so exp/v/spec1.so exp/v/spnolong.so exp/v/nobranch.so exp/v/nocheck.so > gpurun_out/r6i/kp_$c.log 2>&1 || { echo "kp $c failed"; tail -5 gpurun_out/r6i/kp_$c.log; exit 1; }
  grep " us " gpurun_out/r6i/kp_$c.log
done
