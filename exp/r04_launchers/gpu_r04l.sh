#!/bin/bash
set -o pipefail
# Post-parse chain: K_subs 16-byte loads + K_flank 4 bytes/thread + grid-stride
# chunks (j_cur), multi-workgroup mixed-RIGHT sort (k_cur), K_left ablations;
# full-step kernel stats, then the product suite
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out; cd $R
bash scripts/kstats_full_variant.sh kl_k_cur_c3 c3 exp/v/k_cur.so 20 || exit 1
grep -h "RUN ok" gpurun_out/kl_k_cur_c3/log.txt
for c in c4 c5; do
  bash scripts/kstats_full_variant.sh kl_k_cur_$c $c exp/v/k_cur.so 14 || exit 1
done
for v in A_left_noflush A_left_noreads; do
  bash scripts/kstats_full_variant.sh kl_${v}_c3 c3 exp/v/$v.so 6 || exit 1
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t.log 2>&1
rc=$?; echo "product suite:"; tail -2 gpurun_out/t.log; [ $rc -eq 0 ] || { grep -E "^E |Error|FAILED" gpurun_out/t.log | head -20; exit $rc; }
