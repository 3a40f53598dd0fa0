#!/bin/bash
set -o pipefail
# K_left variants: interleaved branch-free slice search (ps), per-gap tally
# word (gw), both; full-step kernel stats at C3 / C4 / C5 / C2
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out; cd $R
for c in ${CONFIGS:-c3 c4 c5 c2}; do
  for v in ${VARIANTS:-l_base l_ps l_gw l_psgw}; do
    bash scripts/kstats_full_variant.sh kl_${v}_$c $c exp/v/$v.so 12 > gpurun_out/kl_${v}_$c.txt 2>&1 || { cat gpurun_out/kl_${v}_$c.txt; exit 1; }
    echo "$c $v $(grep K_left gpurun_out/kl_${v}_$c.txt)"
  done
done
