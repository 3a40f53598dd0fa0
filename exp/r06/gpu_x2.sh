#!/bin/bash
# round 6: 64-bit paired substitution-tally flush -- parity suite with the product, bit-exact check, parse timings
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/x2
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/x2/tests.log 2>&1
rc=$?; grep -E "passed|failed|error" gpurun_out/x2/tests.log | tail -3; [ $rc -eq 0 ] || { grep -E "FAILED|^E " gpurun_out/x2/tests.log | head -20; exit $rc; }
VCHK_CFGS=c1,c2 timeout -k 10 300 python3 -u scripts/variant_check.py exp/v/noflushx2.so exp/v/prod.so > gpurun_out/x2/vchk.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/x2/vchk.log | tail -8; [ $rc -eq 0 ] || exit $rc
for c in c1 c2; do
  KEXP_CFG=$c timeout -k 10 300 python3 -u scripts/kp_multi.py exp/v/noflushx2.so exp/v/prod.so exp/v/noflushx2.so exp/v/prod.so > gpurun_out/x2/kp_$c.log 2>&1 || { echo "kp $c failed"; tail -5 gpurun_out/x2/kp_$c.log; exit 1; }
  grep " us " gpurun_out/x2/kp_$c.log
done
