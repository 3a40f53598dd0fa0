#!/bin/bash
set -o pipefail
# K_parse: L2 touch of the next window before the rounds (MPC_PARSE_L2PF) vs the product, parse phase at C1-C5
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out; cd $R
for c in c2 c3 c5 c4 c1; do
  KEXP_CFG=$c KEXP_ROUNDS=4 timeout -k 10 300 python -u scripts/kp_multi.py exp/v/base.so exp/v/l2pf.so > gpurun_out/kpl2_$c.txt 2>&1 || { tail -20 gpurun_out/kpl2_$c.txt; exit 1; }
  grep "us (rounds" gpurun_out/kpl2_$c.txt
done
