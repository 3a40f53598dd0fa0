#!/bin/bash
# round 6 call C: a variant library through the GPU parity tests, bit-exact vs the round-start library, parse timings
#   bash exp/r06/gpu_c.sh exp/v/<variant>.so [more variants timed]
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/r6c
V=$1
MPC_TEST_LIB=$V timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r6c/tests.log 2>&1
rc=$?; grep -E "passed|failed|error" gpurun_out/r6c/tests.log | tail -3; [ $rc -eq 0 ] || { grep -E "FAILED|^E " gpurun_out/r6c/tests.log | head -20; exit $rc; }
VCHK_CFGS=${VCHK_CFGS:-c1,c2,c4,c5} timeout -k 10 400 python3 -u scripts/variant_check.py exp/v/r5base.so "$@" > gpurun_out/r6c/vchk.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r6c/vchk.log | tail -12; [ $rc -eq 0 ] || exit $rc
for c in ${KP_CFGS:-c2 c3 c5 c4}; do
  KEXP_CFG=$c timeout -k 10 300 python3 -u scripts/kp_multi.py exp/v/r5base.so "$@" > gpurun_out/r6c/kp_$c.log 2>&1 || { echo "kp $c failed"; tail -5 gpurun_out/r6c/kp_$c.log; exit 1; }
  grep " us " gpurun_out/r6c/kp_$c.log
done
