#!/bin/bash
set -o pipefail
# Round-4 experiment call: K_parse variants (exp/v), variant parity, then the product check.
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd $R
for cfg in c2 c3; do
  KEXP_CFG=$cfg timeout -k 10 400 python -u scripts/kparse_only.py exp/v/base.so exp/v/A.so exp/v/A_nodec.so exp/v/A_noeff.so exp/v/A_nodec_noeff.so 2>&1 | tee -a gpurun_out/kp.txt || exit 1
done
KEXP_CFG=c2 timeout -k 10 200 python -u exp/step_time.py exp/v/base.so exp/v/A.so 2>&1 | tee -a gpurun_out/kp.txt || exit 1
MPC_TEST_LIB=exp/v/A.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_depth.py -x -q --timeout 400 --timeout-method thread > gpurun_out/tA.log 2>&1
rc=$?; tail -3 gpurun_out/tA.log; [ $rc -eq 0 ] || { grep -E "^E |Error|FAILED" gpurun_out/tA.log | head -20; exit $rc; }
bash scripts/gpu_r04a.sh
