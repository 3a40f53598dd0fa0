#!/bin/bash
# HBM traffic of K_parse per config (MI355X_MICROARCH.md HBM section: FETCH_SIZE and
# WRITE_SIZE in separate passes, kernel-trace only): bash scripts/pmc_traffic.sh <tag> c2 c3 ...
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp
for c in "$@"; do
  OUT=$R/gpurun_out/${TAG}_$c
  mkdir -p $OUT
  for P in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 200 rocprofv3 --kernel-trace --pmc $P -d $OUT/$P -o run --output-format csv -- \
      python3 $R/bench.py --config $c --steps 2 --warmup 1 --kernel-reps 3 --no-cpu-baseline --no-e2e --hbm-config "" > $OUT/$P.log 2>&1 || { echo "$c $P failed"; tail -5 $OUT/$P.log; exit 1; }
  done
  python3 $R/scripts/traffic.py $OUT K_parse $c $R/gpurun_out/pmc_traffic_$c.json || exit 1
done
