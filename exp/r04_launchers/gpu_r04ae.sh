#!/bin/bash
set -o pipefail
# K_parse epilogue: events per thread per scatter chunk 8 (product) / 12 / 16, parse phase at C1-C5
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out; cd $R
for c in c2 c3 c5 c4 c1; do
  KEXP_CFG=$c KEXP_ROUNDS=4 timeout -k 10 300 python -u scripts/kp_multi.py exp/v/base.so exp/v/epi12.so exp/v/epi16.so > gpurun_out/kpepi_$c.txt 2>&1 || { tail -20 gpurun_out/kpepi_$c.txt; exit 1; }
  grep "us (rounds" gpurun_out/kpepi_$c.txt
done
