#!/bin/bash
# round 5 call B: the full GPU suite with the in-tree library (page-placed
# insertion events), then variants: parity vs head + parse / step timing
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_suite.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_suite.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" gpurun_out/gpu_suite.log | head -20; exit $rc; }
VCHK_CFGS=c1,c2,c4,c5 timeout -k 10 400 python3 -u scripts/variant_check.py exp/v/head.so "$@" > gpurun_out/vchk.log 2>&1
rc=$?; grep -v "^ *$" gpurun_out/vchk.log | tail -30; [ $rc -eq 0 ] || exit $rc
for c in c2 c3 c4 c5 c1; do
  KEXP_CFG=$c timeout -k 10 300 python3 -u scripts/step_multi.py exp/v/head.so "$@" > gpurun_out/stepm_$c.log 2>&1 || { echo "step_multi $c failed"; tail -5 gpurun_out/stepm_$c.log; exit 1; }
  grep " us " gpurun_out/stepm_$c.log
done
