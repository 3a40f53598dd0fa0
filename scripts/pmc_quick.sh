#!/bin/bash
# One PMC pass (SQ instruction mix) over a short bench run: bash scripts/pmc_quick.sh <outname> [config]
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-pmcq}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS \
  -d $OUT/p1 -o run --output-format csv -- python3 $R/bench.py --config ${2:-c2} --steps 2 --warmup 1 --kernel-reps 2 --no-cpu-baseline > $OUT/p1.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS \
  -d $OUT/p2 -o run --output-format csv -- python3 $R/bench.py --config ${2:-c2} --steps 2 --warmup 1 --kernel-reps 2 --no-cpu-baseline > $OUT/p2.log 2>&1
echo rc=$?
