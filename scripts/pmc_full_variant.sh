#!/bin/bash
# LDS / wait counters of one kernel over full pileup steps of a library variant
# (one pass, kernel trace only):  bash scripts/pmc_full_variant.sh <tag> <config> <lib.so> <kernel>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
KEXP_LIB=$R/$3 KEXP_CFG=$2 KEXP_STEPS=3 timeout -s KILL 180 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY \
  -d $OUT/p1 -o run --output-format csv -- python3 $R/scripts/run_child.py > $OUT/p1.log 2>&1 || { echo "pmc failed"; tail -5 $OUT/p1.log; exit 1; }
python3 $R/scripts/pmcsum.py $OUT/p1 $4 | tee $OUT/summary.txt
