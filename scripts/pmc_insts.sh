#!/bin/bash
# SQ instruction / wait counters of K_parse (one pass): bash scripts/pmc_insts.sh <tag> <config>
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_BRANCH SQ_WAIT_INST_ANY \
  -d $OUT/p1 -o run --output-format csv -- python3 $R/bench.py --config ${2:-c2} --steps 2 --warmup 1 --kernel-reps 2 --no-cpu-baseline --no-e2e > $OUT/p1.log 2>&1 || { echo "pmc failed"; tail -5 $OUT/p1.log; exit 1; }
python3 $R/scripts/pmcsum.py $OUT/p1 K_parse | tee $OUT/summary.txt
