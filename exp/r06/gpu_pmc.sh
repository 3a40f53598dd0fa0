#!/bin/bash
# round 6: HBM traffic records (N=1 per config; per-rank shards at N = 2/4/8) and SQ stall counters of the final K_parse
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
bash scripts/pmc_traffic.sh r6p c1 c2 c3 c4 c5 || exit 1
bash scripts/shard_traffic.sh r6p "c1 c2 c3 c4" "2 4 8" || exit 1
bash scripts/pmc_stalls.sh r6s_c3 c3 || exit 1
bash scripts/pmc_stalls.sh r6s_c2 c2 || exit 1
ls gpurun_out/pmc_traffic_*.json
