#!/bin/bash
# full-step timing of exp/v variants: bash exp/run_st.sh "c2 c1" v1 v2 ...
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
CFGS=$1; shift
for c in $CFGS; do
  echo "== step $c"
  libs=""; for v in "$@"; do libs="$libs exp/v/$v.so"; done
  KEXP_CFG=$c timeout -k 10 400 python3 -u exp/step_time.py $libs || exit 1
done
