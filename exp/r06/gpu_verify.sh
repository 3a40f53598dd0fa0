#!/bin/bash
# round 6: the tree as the driver will run it -- smoke and the GPU suite
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r6v}
cd $R && mkdir -p gpurun_out
timeout -k 10 150 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { echo "smoke failed rc=$?"; tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/${TAG}_t.log 2>&1
rc=$?; grep -E "passed|failed|error" gpurun_out/${TAG}_t.log | tail -2
[ $rc -eq 0 ] || { grep -E "FAILED|^E " gpurun_out/${TAG}_t.log | head -30; exit $rc; }
timeout -k 10 300 python3 -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "bench failed"; tail -5 gpurun_out/${TAG}_bench.err; exit 1; }
tail -c 400 gpurun_out/${TAG}_bench.json
