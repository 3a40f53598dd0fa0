#!/bin/bash
set -o pipefail
# K_parse default vs the round's best C5 variant, single-batch kernel stats
# (post-parse chain), E2E at C3 / C5 with the ingest phase split
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out; cd $R
KEXP_CFG=c5 timeout -k 10 300 python -u scripts/kp_multi.py exp/v/h_34.so exp/v/e_default.so > gpurun_out/kpe_c5.txt 2>&1 || { tail -20 gpurun_out/kpe_c5.txt; exit 1; }
grep "us (rounds\|tally_mode" gpurun_out/kpe_c5.txt
bash scripts/kstats_configs.sh r04k c3 c4 c5 || exit 1
for c in c3 c5; do
  MPC_INGEST_TIMING=1 timeout -k 10 400 python -u bench.py --config $c --steps 5 --warmup 2 --kernel-reps 3 --no-cpu-baseline \
    --hbm-config "" > gpurun_out/e2e_$c.log 2> gpurun_out/e2e_$c.err || { tail -20 gpurun_out/e2e_$c.err; exit 1; }
  echo "== e2e $c"; grep -o '"e2e": {.*"write_frac"' gpurun_out/e2e_$c.log | cut -c1-400; grep "^ingest" gpurun_out/e2e_$c.err | tail -12
done
