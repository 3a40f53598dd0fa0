#!/bin/bash
# round 6: deferred placement in tally mode 3 with several substitution windows -- parity, then timing on 20 kb
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/m3
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/m3/tests.log 2>&1
rc=$?; grep -E "passed|failed|error" gpurun_out/m3/tests.log | tail -3; [ $rc -eq 0 ] || { grep -E "FAILED|^E " gpurun_out/m3/tests.log | head -20; exit $rc; }
for sh in 20000,60000 24000,40000; do
  KEXP_SYNTH=$sh timeout -k 10 300 python3 -u scripts/step_multi.py exp/v/prod.so exp/v/nodefer.so exp/v/prod.so exp/v/nodefer.so > gpurun_out/m3/step_$sh.log 2>&1 || { echo "step $sh failed"; tail -5 gpurun_out/m3/step_$sh.log; exit 1; }
  grep " us " gpurun_out/m3/step_$sh.log
done
