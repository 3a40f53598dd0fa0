#!/bin/bash
# rocprofv3 kernel stats of a short bench run per config: bash scripts/kstats_configs.sh <tag> c2 c3 ...
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp
for c in "$@"; do
  OUT=$R/gpurun_out/${TAG}_$c
  mkdir -p $OUT
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- python3 $R/bench.py --config $c --steps 10 --warmup 3 --kernel-reps 3 --no-cpu-baseline --no-e2e --hbm-config "" --inflight ${INFLIGHT:-1} > $OUT/b.log 2>&1 || { echo "$c failed"; tail -5 $OUT/b.log; exit 1; }
  echo "== $c"; python3 $R/scripts/kstats.py $OUT 14
done
