#!/bin/bash
# rocprofv3 kernel stats of full pileup steps of one library variant on one config:
#   bash scripts/kstats_full_variant.sh <tag> <cfg> <lib.so> [n rows]
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; CFG=$2; LIB=$3
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
KEXP_LIB=$R/$LIB KEXP_CFG=$CFG timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- \
  python3 $R/scripts/run_child.py > $OUT/log.txt 2>&1 || { echo "$TAG failed"; tail -5 $OUT/log.txt; exit 1; }
echo "== $TAG ($CFG, $LIB)"; python3 $R/scripts/kstats.py $OUT ${4:-16}
