#!/bin/bash
# SQ instruction / wait counters of K_parse for a library variant (one pass, no
# other tracing):  bash scripts/pmc_variant.sh <tag> <config> <lib.so>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
KEXP_LIB=$R/$3 KEXP_CFG=$2 KEXP_REPS=3 timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_BRANCH SQ_WAIT_INST_ANY \
  -d $OUT/p1 -o run --output-format csv -- python3 $R/scripts/kp_child.py > $OUT/p1.log 2>&1 || { echo "pmc failed"; tail -5 $OUT/p1.log; exit 1; }
python3 $R/scripts/pmcsum.py $OUT/p1 K_parse | tee $OUT/summary.txt
