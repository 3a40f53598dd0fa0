#!/bin/bash
# round 6 measurements with the product kernels: smoke, the GPU suite, bench lines + rocprofv3 kernel stats per config
#   bash exp/r06/gpu_final.sh <tag>
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r6f}
cd $R && mkdir -p gpurun_out
timeout -k 10 150 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { echo "smoke failed rc=$?"; tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/${TAG}_t.log 2>&1
rc=$?; grep -E "passed|failed|error" gpurun_out/${TAG}_t.log | tail -2
[ $rc -eq 0 ] || { grep -E "FAILED|^E " gpurun_out/${TAG}_t.log | head -30; exit $rc; }
bash $R/scripts/final_configs.sh $TAG c2 c1 c3 c4 c5
