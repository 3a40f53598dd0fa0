#!/bin/bash
set -o pipefail
# K_flank loop shape (bytes per thread) x grid (grid-stride chunks) at C3,
# then LDS counters of K_left and K_flank at C3
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out; cd $R
for c in c3; do
  for v in fl_b1_ginf fl_b4_ginf fl_b1_g1024 fl_b4_g1024 fl_b1_g2048; do
    bash scripts/kstats_full_variant.sh km_${v}_$c $c exp/v/$v.so 40 | grep -E "==|K_flank" || exit 1
  done
done
bash scripts/pmc_full_variant.sh pm_left_c3 c3 exp/v/fl_b1_ginf.so K_left || exit 1
bash scripts/pmc_full_variant.sh pm_flank_c3 c3 exp/v/fl_b1_ginf.so K_flank || exit 1
