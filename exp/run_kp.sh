#!/bin/bash
# parse-only timing of exp/v variants at the given configs: bash exp/run_kp.sh "c2 c4" v1 v2 ...
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
CFGS=$1; shift
for c in $CFGS; do
  echo "== $c"
  libs=""; for v in "$@"; do libs="$libs exp/v/$v.so"; done
  KEXP_CFG=$c timeout -k 10 400 python3 -u scripts/kparse_only.py $libs || exit 1
done
