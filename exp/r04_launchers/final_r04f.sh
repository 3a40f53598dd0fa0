#!/bin/bash
set -o pipefail
# end-of-round check on the committed tree: smoke, the GPU suite, the default bench line
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/f4f_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/f4f_smoke.log; exit 1; }
tail -1 gpurun_out/f4f_smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/f4f_t.log 2>&1
rc=$?; grep -E "passed|failed|error" gpurun_out/f4f_t.log | tail -2; [ $rc -eq 0 ] || { grep -E "FAILED|^E " gpurun_out/f4f_t.log | head -30; exit $rc; }
timeout -k 10 400 python3 -u bench.py > gpurun_out/f4f_c2.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/f4f_c2.log; exit 1; }
grep '^{' gpurun_out/f4f_c2.log | tail -1 > gpurun_out/f4f_c2_bench.json; cut -c1-250 gpurun_out/f4f_c2_bench.json
