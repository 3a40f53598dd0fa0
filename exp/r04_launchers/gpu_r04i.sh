#!/bin/bash
set -o pipefail
# K_rsort stage ablations at C3 (no sort passes, no value gather) and K_flank
# without its per-byte tallies; full-step kernel stats
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out; cd $R
for v in g_default A_rsort_nopass A_rsort_novals A_flank_nobytes; do
  bash scripts/kstats_full_variant.sh kg_${v}_c3 c3 exp/v/$v.so 8 || exit 1
done
