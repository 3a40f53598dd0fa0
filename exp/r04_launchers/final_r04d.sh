#!/bin/bash
set -o pipefail
# C1 bench line with its new default (4 batches in flight, parse grid on 96 CUs)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python3 -u bench.py --config c1 > gpurun_out/f4d_c1.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/f4d_c1.log; exit 1; }
grep '^{' gpurun_out/f4d_c1.log | tail -1 > gpurun_out/f4d_c1_bench.json; cut -c1-300 gpurun_out/f4d_c1_bench.json
