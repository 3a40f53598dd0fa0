#!/bin/bash
# smoke, the full -m gpu suite, then bench lines of the given configs
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 180 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_suite.log 2>&1
rc=$?; tail -2 gpurun_out/gpu_suite.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" gpurun_out/gpu_suite.log | head -20; exit $rc; }
if [ $# -gt 0 ]; then bash exp/r05/bench_lines.sh "$@"; fi
