#!/bin/bash
set -o pipefail
# K_subs with 16-byte event loads (+ K_subsum row groups), K_flank 4 bytes per
# thread (i_cur: both): kernel stats, then the product suite
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out; cd $R
for c in c3 c4 c5; do
  bash scripts/kstats_full_variant.sh kh_i_cur_$c $c exp/v/i_cur.so 14 || exit 1
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t.log 2>&1
rc=$?; echo "product suite:"; tail -2 gpurun_out/t.log; [ $rc -eq 0 ] || { grep -E "^E |Error|FAILED" gpurun_out/t.log | head -20; exit $rc; }
