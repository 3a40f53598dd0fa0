#!/bin/bash
# round 6: K_left runs counted before the tally (MPC_LEFT_KQ) -- parity suite, bit-exact check, full steps
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/kq
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/kq/tests.log 2>&1
rc=$?; grep -E "passed|failed|error" gpurun_out/kq/tests.log | tail -3; [ $rc -eq 0 ] || { grep -E "FAILED|^E " gpurun_out/kq/tests.log | head -20; exit $rc; }
VCHK_CFGS=c2,c3,c4,c5 timeout -k 10 400 python3 -u scripts/variant_check.py exp/v/nokq.so exp/v/prod.so > gpurun_out/kq/vchk.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/kq/vchk.log | tail -8; [ $rc -eq 0 ] || exit $rc
bash exp/r06/gpu_step.sh "c3 c4 c2 c5" exp/v/prod.so exp/v/nokq.so exp/v/prod.so exp/v/nokq.so
