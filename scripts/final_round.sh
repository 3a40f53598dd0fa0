#!/bin/bash
# Round-end measurements in one call: smoke, the GPU suite, then per config the
# full bench line (CPU baseline, E2E, C3 HBM roofline) and rocprofv3 kernel stats:
#   bash scripts/final_round.sh <tag> c2 c1 c3 c4 c5
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
cd $R && mkdir -p gpurun_out
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { echo "smoke failed rc=$?"; tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${TAG}_t.log 2>&1
rc=$?
grep -E "passed|failed|error" gpurun_out/${TAG}_t.log | tail -2
[ $rc -eq 0 ] || { grep -E "FAILED|^E " gpurun_out/${TAG}_t.log | head -30; exit $rc; }
bash $R/scripts/final_configs.sh $TAG "$@"
