#!/bin/bash
# GPU test suite (one process), then rocprofv3 kernel stats of the given configs:
#   bash scripts/gpu_tests_kstats.sh <tag> c2 c3 ...
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
cd $R && mkdir -p gpurun_out
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { echo "smoke failed rc=$?"; tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${TAG}_t.log 2>&1
rc=$?
grep -E "passed|failed|error" gpurun_out/${TAG}_t.log | tail -3
[ $rc -eq 0 ] || { grep -E "FAILED|^E " gpurun_out/${TAG}_t.log | head -30; exit $rc; }
bash $R/scripts/kstats_configs.sh $TAG "$@"
