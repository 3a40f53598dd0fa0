#!/bin/bash
# round 6 call M: product with deferred placement -- smoke, GPU suite, bench lines per config, then
# parse-phase timings against the library without it (exp/v/nodefer.so), bit-exact check first
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r6d}
cd $R && mkdir -p gpurun_out/$TAG
bash exp/r06/gpu_final.sh $TAG || exit 1
VCHK_CFGS=c2,c3,c4 timeout -k 10 400 python3 -u scripts/variant_check.py exp/v/r5base.so exp/v/prod.so exp/v/nodefer.so > gpurun_out/$TAG/vchk.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/$TAG/vchk.log | tail -8; [ $rc -eq 0 ] || exit $rc
for c in c2 c3 c4; do
  KEXP_CFG=$c timeout -k 10 300 python3 -u scripts/kp_multi.py exp/v/nodefer.so exp/v/prod.so exp/v/nodefer.so exp/v/prod.so > gpurun_out/$TAG/kp_$c.log 2>&1 || { echo "kp $c failed"; tail -5 gpurun_out/$TAG/kp_$c.log; exit 1; }
  grep " us " gpurun_out/$TAG/kp_$c.log
done
