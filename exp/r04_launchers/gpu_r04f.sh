#!/bin/bash
set -o pipefail
# K_parse read-base variants (LDS round trip vs scalar pass per tally mode), DMA off,
# then the product suite, the default bench line and K_parse stamps
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out; cd $R
V="exp/v/base.so exp/v/h_34.so exp/v/d_default.so exp/v/d_noldsbase.so exp/v/d_allldsbase.so"
for c in c2 c1 c3 c5; do
  KEXP_CFG=$c timeout -k 10 300 python -u scripts/kp_multi.py $V > gpurun_out/kpd_$c.txt 2>&1 || { tail -20 gpurun_out/kpd_$c.txt; exit 1; }
  grep "us (rounds" gpurun_out/kpd_$c.txt
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t.log 2>&1
rc=$?; echo "product suite:"; tail -2 gpurun_out/t.log; [ $rc -eq 0 ] || { grep -E "^E |Error|FAILED" gpurun_out/t.log | head -20; exit $rc; }
timeout -k 10 300 python -u bench.py > gpurun_out/b.log 2> gpurun_out/b.err || { tail -20 gpurun_out/b.err; exit 1; }
tail -1 gpurun_out/b.log | cut -c1-300
timeout -k 10 300 python -u scripts/kparse_stamps.py exp/v/stamps.so c2 c3 > gpurun_out/stamps.txt 2>&1 || { tail -20 gpurun_out/stamps.txt; exit 1; }
cat gpurun_out/stamps.txt | grep -v amdgpu.ids
