#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/r6g
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -q -k "two_byte or mixed" --timeout 120 --timeout-method thread > gpurun_out/r6g/t_product.log 2>&1
rc=$?; tail -2 gpurun_out/r6g/t_product.log; [ $rc -eq 0 ] || exit $rc
MPC_TEST_LIB=exp/v/r5base.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -q -k "two_byte" --timeout 120 --timeout-method thread > gpurun_out/r6g/t_r5base.log 2>&1
echo "round-5 library on the two-byte test: rc=$?"; grep -E "passed|failed|differs" gpurun_out/r6g/t_r5base.log | head -3
for c in c3 c5 c2; do
  KEXP_CFG=$c timeout -k 10 300 python3 -u scripts/kp_multi.py exp/v/base.so exp/v/nobranch.so exp/v/leanforce.so exp/v/nocheck.so > gpurun_out/r6g/kp_$c.log 2>&1 || { echo "kp $c failed"; tail -5 gpurun_out/r6g/kp_$c.log; exit 1; }
  grep " us " gpurun_out/r6g/kp_$c.log
done
