#!/bin/bash
set -o pipefail
# Post-parse experiments: K_subs slab + K_subsum vs global-atomic flush vs no
# flush (ablation), K_flank window flush ablation; full-step kernel stats
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out; cd $R
for c in c3 c4 c5; do
  for v in f_slab f_atomic A_subs_noflush A_flank_noflush; do
    bash scripts/kstats_full_variant.sh kf_${v}_$c $c exp/v/$v.so 12 || exit 1
  done
done
grep -h "RUN ok" gpurun_out/kf_f_slab_c*/log.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t.log 2>&1
rc=$?; echo "product suite:"; tail -2 gpurun_out/t.log; [ $rc -eq 0 ] || { grep -E "^E |Error|FAILED" gpurun_out/t.log | head -20; exit $rc; }
