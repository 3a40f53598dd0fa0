#!/bin/bash
set -o pipefail
# K_parse variants (fast decode per tally mode, LDS-DMA staging) on c1..c5,
# then the product suite, the C2 bench line and E2E with the ingest phase split
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out; cd $R
V="exp/v/base.so exp/v/v4f.so exp/v/h_all_dma.so exp/v/h_all.so exp/v/h_none.so exp/v/h_34.so exp/v/h_none_dma.so"
for c in c2 c3 c4 c5 c1; do
  KEXP_CFG=$c timeout -k 10 300 python -u scripts/kp_multi.py $V > gpurun_out/kpm_$c.txt 2>&1 || { tail -20 gpurun_out/kpm_$c.txt; exit 1; }
  grep "us (rounds" gpurun_out/kpm_$c.txt
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t.log 2>&1
rc=$?; echo "product suite:"; tail -2 gpurun_out/t.log; [ $rc -eq 0 ] || { grep -E "^E |Error|FAILED" gpurun_out/t.log | head -20; exit $rc; }
MPC_INGEST_TIMING=1 timeout -k 10 300 python -u bench.py --hbm-config c3 > gpurun_out/b.log 2> gpurun_out/b.err || { tail -20 gpurun_out/b.err; exit 1; }
tail -1 gpurun_out/b.log | cut -c1-600; grep "^ingest" gpurun_out/b.err | tail -8
MPC_INGEST_TIMING=1 timeout -k 10 400 python -u bench.py --config c3 --steps 5 --warmup 2 --kernel-reps 3 --no-cpu-baseline \
  --hbm-config "" > gpurun_out/e2e_c3.log 2> gpurun_out/e2e_c3.err || { tail -20 gpurun_out/e2e_c3.err; exit 1; }
grep -o '"e2e": {.*"what"' gpurun_out/e2e_c3.log | cut -c1-400; grep "^ingest" gpurun_out/e2e_c3.err | tail -12
