#!/bin/bash
set -o pipefail
# Multi-workgroup mixed-RIGHT sort (k_cur) at C3, then the product suite
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out; cd $R
bash scripts/kstats_full_variant.sh kk_k_cur_c3 c3 exp/v/k_cur.so 20 || exit 1
grep -h "RUN ok" gpurun_out/kk_k_cur_c3/log.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t.log 2>&1
rc=$?; echo "product suite:"; tail -2 gpurun_out/t.log; [ $rc -eq 0 ] || { grep -E "^E |Error|FAILED" gpurun_out/t.log | head -20; exit $rc; }
for v in A_left_noflush A_left_noreads; do
  bash scripts/kstats_full_variant.sh kk_${v}_c3 c3 exp/v/$v.so 6 || exit 1
done
