#!/bin/bash
# parity tests + per-kernel timing of the in-tree library (and any variants given as args)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1
rc=$?
tail -3 gpurun_out/t.log
[ $rc -eq 0 ] || { grep -E "^E |Error|FAIL" gpurun_out/t.log | head -30; exit $rc; }
timeout -k 10 300 python3 scripts/kexp.py minion-plasmid-consensus_amd/libmpc.so "$@"
