#!/bin/bash
# Per-rank step of an N-GPU run predicted on one GPU:
# all N shards of one global read set stepped in-process (scripts/shard_probe.py
# --mode step), rocprofv3 kernel stats -> gpurun_out/<tag>_<cfg>_w<N>/
#   bash scripts/shard_step.sh <tag> "c3" "8"
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; CFGS=$2; WORLDS=$3
cd /tmp && export TMPDIR=/tmp
for c in $CFGS; do
  for w in $WORLDS; do
    OUT=$R/gpurun_out/${TAG}_${c}_w$w
    mkdir -p $OUT
    timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- \
      python3 $R/scripts/shard_probe.py --config $c --world $w --mode step --reps 5 > $OUT/probe.log 2>&1 \
      || { echo "$c w$w failed"; tail -5 $OUT/probe.log; exit 1; }
  done
done
