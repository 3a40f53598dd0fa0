#!/bin/bash
# Per-rank K_parse HBM traffic of N-GPU runs, measured on one GPU (VERDICT r05
# item 5a): rank 0's shard of the N-shard plan (scripts/shard_probe.py --mode
# parse), FETCH_SIZE and WRITE_SIZE in separate rocprofv3 passes (the MI355X
# guide's HBM recipe, scripts/traffic.py) -> gpurun_out/pmc_traffic_<cfg>_w<N>.json
#   bash scripts/shard_traffic.sh <tag> "c2 c3" "2 4 8"
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; CFGS=$2; WORLDS=$3
cd /tmp && export TMPDIR=/tmp
for c in $CFGS; do
  for w in $WORLDS; do
    OUT=$R/gpurun_out/${TAG}_${c}_w$w
    mkdir -p $OUT
    for P in FETCH_SIZE WRITE_SIZE; do
      timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $P -d $OUT/$P -o run --output-format csv -- \
        python3 $R/scripts/shard_probe.py --config $c --world $w --mode parse --reps 4 > $OUT/$P.log 2>&1 \
        || { echo "$c w$w $P failed"; tail -5 $OUT/$P.log; exit 1; }
    done
    python3 $R/scripts/traffic.py $OUT K_parse $c $R/gpurun_out/pmc_traffic_${c}_w$w.json $w || exit 1
  done
done
