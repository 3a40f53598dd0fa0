#!/bin/bash
set -o pipefail
# K_parse with its effects removed (decode + one packed word per unit): the
# pass-1 cost of a tokenize / effects split, against the product kernel; then
# the GPU suite on the final tree
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out; cd $R
for c in c3 c2 c4; do
  KEXP_CFG=$c timeout -k 10 300 python -u scripts/kp_multi.py exp/v/fl_b1_ginf.so exp/v/A_tokenize.so > gpurun_out/kpq_$c.txt 2>&1 || { tail -20 gpurun_out/kpq_$c.txt; exit 1; }
  grep "us (rounds" gpurun_out/kpq_$c.txt
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t.log 2>&1
rc=$?; echo "product suite:"; tail -2 gpurun_out/t.log; [ $rc -eq 0 ] || { grep -E "^E |Error|FAILED" gpurun_out/t.log | head -20; exit $rc; }
