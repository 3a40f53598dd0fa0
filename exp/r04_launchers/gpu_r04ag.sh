#!/bin/bash
set -o pipefail
# batches in flight with parse / post-parse chain on CU-masked streams (exp/cusplit.py)
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out; cd $R
timeout -k 10 300 python3 -u exp/cusplit.py c2 3 run split mask:4 mask:8 run > gpurun_out/cusplit_c2.txt 2>&1 || { tail -20 gpurun_out/cusplit_c2.txt; exit 1; }
grep "per step" gpurun_out/cusplit_c2.txt
timeout -k 10 200 python3 -u exp/cusplit.py c1 4 run split mask:4 mask:8 > gpurun_out/cusplit_c1.txt 2>&1 || { tail -20 gpurun_out/cusplit_c1.txt; exit 1; }
grep "per step" gpurun_out/cusplit_c1.txt
