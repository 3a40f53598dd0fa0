#!/bin/bash
# round 6 call B: split rounds -- bit-exact vs the round-start library, parse timings
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/r6b
VCHK_CFGS=${VCHK_CFGS:-c1,c2,c4,c5} timeout -k 10 400 python3 -u scripts/variant_check.py exp/v/r5base.so "$@" > gpurun_out/r6b/vchk.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r6b/vchk.log | tail -12; [ $rc -eq 0 ] || exit $rc
for c in ${KP_CFGS:-c2 c3 c5 c4}; do
  KEXP_CFG=$c timeout -k 10 300 python3 -u scripts/kp_multi.py exp/v/r5base.so "$@" > gpurun_out/r6b/kp_$c.log 2>&1 || { echo "kp $c failed"; tail -5 gpurun_out/r6b/kp_$c.log; exit 1; }
  grep " us " gpurun_out/r6b/kp_$c.log
done
