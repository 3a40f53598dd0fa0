#!/bin/bash
set -o pipefail
# smoke + the whole GPU suite on the current tree
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/f4e_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/f4e_smoke.log; exit 1; }
tail -1 gpurun_out/f4e_smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/f4e_t.log 2>&1
rc=$?; grep -E "passed|failed|error" gpurun_out/f4e_t.log | tail -2; [ $rc -eq 0 ] || { grep -E "FAILED|^E " gpurun_out/f4e_t.log | head -30; exit $rc; }
