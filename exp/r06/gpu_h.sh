#!/bin/bash
# round 6 call H: the speculative parse as the product -- parity tests, how often it falls back, parse timings
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/r6h
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_depth.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r6h/tests.log 2>&1
rc=$?; grep -E "passed|failed|error" gpurun_out/r6h/tests.log | tail -2; [ $rc -eq 0 ] || { grep -E "FAILED|^E " gpurun_out/r6h/tests.log | head -20; exit $rc; }
timeout -k 10 300 python3 -u exp/r06/spec_diag.py c1 c2 c3 c4 c5 > gpurun_out/r6h/spec.log 2>&1; rc=$?; grep spec_failed gpurun_out/r6h/spec.log; [ $rc -eq 0 ] || exit $rc
for c in c2 c3 c5 c4 c1; do
  KEXP_CFG=$c timeout -k 10 300 python3 -u scripts/kp_multi.py exp/v/r5base.so exp/v/base.so exp/v/nospec.so exp/v/nocheck.so > gpurun_out/r6h/kp_$c.log 2>&1 || { echo "kp $c failed"; tail -5 gpurun_out/r6h/kp_$c.log; exit 1; }
  grep " us " gpurun_out/r6h/kp_$c.log
done
