#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/r6l
MPC_TEST_LIB=exp/v/m12opt.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r6l/tests.log 2>&1
rc=$?; grep -E "passed|failed|error" gpurun_out/r6l/tests.log | tail -2; [ $rc -eq 0 ] || { grep -E "FAILED|^E " gpurun_out/r6l/tests.log | head -20; exit $rc; }
VCHK_CFGS=c1,c2 timeout -k 10 300 python3 -u scripts/variant_check.py exp/v/prod.so exp/v/m12opt.so > gpurun_out/r6l/vchk.log 2>&1; rc=$?; grep "==\|differ" gpurun_out/r6l/vchk.log | tail -4; [ $rc -eq 0 ] || exit $rc
for c in c2 c1 c2; do
  KEXP_CFG=$c KEXP_ROUNDS=5 timeout -k 10 300 python3 -u scripts/kp_multi.py exp/v/prod.so exp/v/m12opt.so > gpurun_out/r6l/kp_$c.log 2>&1 || { echo "kp $c failed"; exit 1; }
  grep " us " gpurun_out/r6l/kp_$c.log
done
