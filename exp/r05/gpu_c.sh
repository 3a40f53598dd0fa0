#!/bin/bash
# round 5 call C: variants parity vs head + parse / step timing (no suite)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
VCHK_CFGS=${VCHK_CFGS:-c1,c2,c4,c5} timeout -k 10 400 python3 -u scripts/variant_check.py exp/v/head.so "$@" > gpurun_out/vchk.log 2>&1
rc=$?; grep -v "^ *$" gpurun_out/vchk.log | grep -v amdgpu.ids | tail -30; [ $rc -eq 0 ] || exit $rc
for c in ${STEP_CFGS:-c2 c3 c4 c5 c1}; do
  KEXP_CFG=$c timeout -k 10 300 python3 -u scripts/step_multi.py exp/v/head.so "$@" > gpurun_out/stepm_$c.log 2>&1 || { echo "step_multi $c failed"; tail -5 gpurun_out/stepm_$c.log; exit 1; }
  grep " us " gpurun_out/stepm_$c.log
done
