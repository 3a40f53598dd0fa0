#!/bin/bash
# one-kernel timing of exp/v variants: bash exp/run_k.sh kernel "c2 c3" v1 v2 ...
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
K=$1; CFGS=$2; shift 2
for c in $CFGS; do
  echo "== $K $c"
  libs=""; for v in "$@"; do libs="$libs exp/v/$v.so"; done
  KEXP_KERNEL=$K KEXP_CFG=$c timeout -k 10 400 python3 -u scripts/kernel_only.py $libs || exit 1
done
