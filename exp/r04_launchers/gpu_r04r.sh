#!/bin/bash
set -o pipefail
# K_left: per-segment stamps (diagnostic build) on C3/C4/C5/C2, then full-step
# kernel stats of the next-unit record prefetch against the base build
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out; cd $R
timeout -k 10 300 python3 -u scripts/kleft_stamps.py exp/v/lstamps.so c3 c4 c5 c2 > gpurun_out/kleft_stamps.txt 2>&1 || { tail -20 gpurun_out/kleft_stamps.txt; exit 1; }
cat gpurun_out/kleft_stamps.txt
for c in c3 c5; do
  for v in l_base l_pf; do
    bash scripts/kstats_full_variant.sh kl_${v}_$c $c exp/v/$v.so 6 || exit 1
  done
done
