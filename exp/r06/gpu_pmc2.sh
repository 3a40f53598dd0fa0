#!/bin/bash
# round 6, after deferred placement: HBM traffic records of the configs whose K_parse changed (C2-C4; N = 1 and
# per-rank shards at N = 2/4/8) and SQ stall / instruction counters at C3 and C2
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
bash scripts/pmc_traffic.sh r6q c2 c3 c4 || exit 1
bash scripts/shard_traffic.sh r6q "c2 c3 c4" "2 4 8" || exit 1
bash scripts/pmc_stalls.sh r6t_c3 c3 || exit 1
bash scripts/pmc_stalls.sh r6t_c2 c2 || exit 1
ls gpurun_out/pmc_traffic_*.json
