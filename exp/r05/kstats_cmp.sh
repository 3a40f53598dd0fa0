#!/bin/bash
# rocprofv3 kernel stats of variants per config: bash exp/r05/kstats_cmp.sh "c2 c5" exp/v/a.so exp/v/b.so
R=${GRAFT_REPO_ROOT:-$(pwd)}
CFGS=$1; shift
cd /tmp && export TMPDIR=/tmp
for CFG in $CFGS; do
for lib in "$@"; do
  n=$(basename $lib .so)
  OUT=$R/gpurun_out/ks_${CFG}_$n
  mkdir -p $OUT
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- python3 $R/exp/var_steps.py $R/$lib $CFG 12 > $OUT/b.log 2>&1 || { echo "$n failed"; tail -5 $OUT/b.log; exit 1; }
  echo "== $CFG $n"; python3 $R/scripts/kstats.py $OUT 14
done
done
