#!/bin/bash
# K_parse HBM traffic (FETCH_SIZE / WRITE_SIZE, separate passes) of library
# variants on one config:  bash scripts/traffic_variant.sh <tag> <config> a.so b.so ...
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; CFG=$2; shift 2
cd /tmp && export TMPDIR=/tmp
for L in "$@"; do
  V=$(basename $L .so)
  OUT=$R/gpurun_out/${TAG}_${CFG}_$V
  mkdir -p $OUT
  for P in FETCH_SIZE WRITE_SIZE; do
    KEXP_LIB=$R/$L KEXP_CFG=$CFG KEXP_REPS=3 timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $P -d $OUT/$P -o run \
      --output-format csv -- python3 $R/scripts/kp_child.py > $OUT/$P.log 2>&1 || { echo "$V $P failed"; tail -5 $OUT/$P.log; exit 1; }
  done
  python3 $R/scripts/traffic.py $OUT K_parse $CFG $OUT/traffic.json > /dev/null || exit 1
  python3 -c "import json; d=json.load(open('$OUT/traffic.json')); print('$CFG $V fetch %.1f MB write %.1f MB' % (d['fetch_bytes_per_launch']/1e6, d['write_bytes_per_launch']/1e6))"
done
