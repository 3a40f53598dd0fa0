#!/bin/bash
# SQ instruction mix / waits / LDS conflicts of every kernel on one config: bash scripts/pmc_kernels.sh <tag> <config> [kernel-substrings...]
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
CFG=$2; shift 2
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT \
  -d $OUT/p1 -o run --output-format csv -- python3 $R/bench.py --config $CFG --steps 2 --warmup 1 --kernel-reps 2 --no-cpu-baseline --no-e2e > $OUT/p1.log 2>&1 || { echo "pass 1 failed"; tail -5 $OUT/p1.log; exit 1; }
timeout -k 10 240 rocprofv3 --kernel-trace --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH SQ_BUSY_CYCLES \
  -d $OUT/p2 -o run --output-format csv -- python3 $R/bench.py --config $CFG --steps 2 --warmup 1 --kernel-reps 2 --no-cpu-baseline --no-e2e > $OUT/p2.log 2>&1 || { echo "pass 2 failed"; tail -5 $OUT/p2.log; exit 1; }
python3 $R/scripts/pmcsum.py $OUT "$@"
