#!/bin/bash
# round 6 call A: nocheck bit-exactness on synthetic configs, parse timings, C5 write counters per variant
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/r6a
VCHK_CFGS=c2,c5 timeout -k 10 300 python3 -u scripts/variant_check.py exp/v/base.so exp/v/nocheck.so > gpurun_out/r6a/vchk.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r6a/vchk.log | tail -6; [ $rc -eq 0 ] || exit $rc
for c in c2 c3 c5; do
  KEXP_CFG=$c timeout -k 10 300 python3 -u scripts/kp_multi.py exp/v/base.so exp/v/nocheck.so exp/v/subnt.so > gpurun_out/r6a/kp_$c.log 2>&1 || { echo "kp $c failed"; tail -5 gpurun_out/r6a/kp_$c.log; exit 1; }
  grep " us " gpurun_out/r6a/kp_$c.log
done
bash scripts/traffic_variant.sh r6a c5 exp/v/base.so exp/v/noevstore.so exp/v/nosubstore.so exp/v/subnt.so
