#!/bin/bash
set -o pipefail
# K_subs: slab + K_subsum vs global-atomic flush (and the flush ablation), kernel stats of the parse phase
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out; cd $R
for c in c3 c4 c5; do
  for v in f_slab f_atomic A_subs_noflush; do
    bash scripts/kstats_variant.sh ks_${v}_$c $c exp/v/$v.so || exit 1
  done
done
