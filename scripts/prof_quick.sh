#!/bin/bash
# kernel stats + one SQ PMC pass on a short bench run: bash scripts/prof_quick.sh <name> <config> [lib]
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
CFG=${2:-c2}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/ks -o run --output-format csv -- python3 $R/bench.py --config $CFG --steps 5 --warmup 2 --kernel-reps 3 --no-cpu-baseline --no-e2e > $OUT/ks.log 2>&1 || { echo "ks failed"; tail -5 $OUT/ks.log; exit 1; }
python3 $R/scripts/kstats.py $OUT/ks 14
timeout -k 10 240 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD \
  -d $OUT/p1 -o run --output-format csv -- python3 $R/bench.py --config $CFG --steps 2 --warmup 1 --kernel-reps 2 --no-cpu-baseline --no-e2e > $OUT/p1.log 2>&1 || { echo "pmc failed"; tail -5 $OUT/p1.log; exit 1; }
python3 $R/scripts/pmcsum.py $OUT/p1 K_parse K_lanes
