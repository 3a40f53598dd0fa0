#!/bin/bash
# round 5 call A: golden CLI parity (new negative-tstart cases) with the in-tree
# library, then K_parse variants (parity vs head + timing)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "cli_matches or max_reference or many_reads" > gpurun_out/golden.log 2>&1
rc=$?; tail -3 gpurun_out/golden.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/golden.log | head -20; exit $rc; }
bash exp/r05/kp_variants.sh "$@"
