#!/bin/bash
set -o pipefail
# K_flank grid / loop shape at C3 and the LDS counters of K_left
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out; cd $R
for v in fl_b1_ginf fl_b1_g1024 fl_b4_g1024; do
  bash scripts/kstats_full_variant.sh km_${v}_c3 c3 exp/v/$v.so 40 | grep -E "==|K_flank" || exit 1
done
bash scripts/pmc_full_variant.sh pm_left_c3 c3 exp/v/fl_b1_ginf.so K_left || exit 1
timeout -k 10 200 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29541 \
  exp/dist_overhead.py c2 2>&1 | grep -v "^\[W\|Warning" | tee gpurun_out/dist_overhead.txt || exit 1
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29543 \
  bench.py --dist --graph --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --hbm-config '' > gpurun_out/bdg.log 2>&1 || { tail -20 gpurun_out/bdg.log; exit 1; }
grep '^{' gpurun_out/bdg.log | tail -1 | cut -c1-200; grep -o '"graph": "[^"]*"' gpurun_out/bdg.log
bash scripts/pmc_traffic.sh f4pmc c2 c3 || exit 1
cat gpurun_out/pmc_traffic_c2.json gpurun_out/pmc_traffic_c3.json
