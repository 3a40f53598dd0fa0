#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/r6e
timeout -k 10 300 python3 -u exp/r06/lean_diag.py exp/v/leandiag.so c2 c3 c5 > gpurun_out/r6e/diag.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/r6e/diag.log | tail -5; [ $rc -eq 0 ] || exit $rc
for c in c3 c2; do
  KEXP_CFG=$c timeout -k 10 300 python3 -u scripts/kp_multi.py exp/v/nosplit.so exp/v/leanforce.so exp/v/nocheck.so exp/v/lean2.so > gpurun_out/r6e/kp_$c.log 2>&1 || { echo "kp $c failed"; tail -5 gpurun_out/r6e/kp_$c.log; exit 1; }
  grep " us " gpurun_out/r6e/kp_$c.log
done
