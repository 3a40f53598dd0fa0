#!/bin/bash
# in-flight step time of variant builds (sensitivity of the C2 bench to one kernel):
#   PARSE_CUS=192 bash exp/r05/sens.sh c2 3 exp/v/a.so exp/v/b.so ...
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
CFG=$1; IF=$2; shift 2
for rep in 1 2; do
for lib in "$@"; do
  n=$(basename $lib .so)
  KEXP_LIB=$lib timeout -k 10 200 python3 -u exp/overlap.py $CFG $IF > gpurun_out/sens_${CFG}_$n.log 2>&1 || { echo "$n failed"; tail -5 gpurun_out/sens_${CFG}_$n.log; exit 1; }
  echo "rep$rep $n cus=$PARSE_CUS: $(grep 'us per step' gpurun_out/sens_${CFG}_$n.log)"
done
done
