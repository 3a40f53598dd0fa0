#!/bin/bash
set -o pipefail
# K_parse grid size (workgroups; 256 = one per CU, the planner's default) at C3 / C4 / C5 / C2
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out; cd $R
for c in c3 c2 c5 c4; do
  KEXP_CFG=$c timeout -k 10 300 python3 -u scripts/kp_wgs.py exp/v/tune.so 256 512 768 1024 2048 > gpurun_out/kpwgs_$c.txt 2>&1 || { tail -5 gpurun_out/kpwgs_$c.txt; exit 1; }
  grep -v amdgpu.ids gpurun_out/kpwgs_$c.txt
done
