#!/bin/bash
# variants of K_parse: parity against the product library, then parse-phase timing per config
# bash exp/r05/kp_variants.sh "cfgs for check" "cfgs for timing" lib1 lib2 ...
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
CHK=$1; TIM=$2; shift 2
V="$@"
VCHK_CFGS=$CHK timeout -k 10 400 python3 -u scripts/variant_check.py exp/v/head.so $V > gpurun_out/vchk.log 2>&1
rc=$?; cat gpurun_out/vchk.log | grep -v "^ *$" | tail -30
[ $rc -eq 0 ] || exit $rc
for c in ${TIM//,/ }; do
  KEXP_CFG=$c KEXP_ROUNDS=3 KEXP_REPS=10 timeout -k 10 300 python3 -u scripts/kp_multi.py exp/v/head.so $V > gpurun_out/kpm_$c.log 2>&1 || { echo "kp_multi $c failed"; tail -5 gpurun_out/kpm_$c.log; exit 1; }
  grep " us " gpurun_out/kpm_$c.log
done
