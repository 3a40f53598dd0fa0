#!/bin/bash
# rocprofv3 kernel stats of library variants: bash exp/var_kstats.sh <tag> <cfg> exp/v/a.so exp/v/b.so ...
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; CFG=$2; shift 2
cd /tmp && export TMPDIR=/tmp
for lib in "$@"; do
  n=$(basename $lib .so)
  OUT=$R/gpurun_out/${TAG}_${CFG}_$n
  mkdir -p $OUT
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- python3 $R/exp/var_steps.py $R/$lib $CFG 12 > $OUT/b.log 2>&1 || { echo "$n failed"; tail -5 $OUT/b.log; exit 1; }
  echo "== $CFG $n"; python3 $R/scripts/kstats.py $OUT 16 | grep -E "K_layout|K_select|K_call"
done
