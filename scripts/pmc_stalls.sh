#!/bin/bash
# Stall attribution of the parse kernel: SQ issue / wait / LDS counters, one
# rocprofv3 --pmc pass per counter group (kernel-trace only, no other domains).
#   bash scripts/pmc_stalls.sh <tag> <config> [kernel-substring]
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
CFG=${2:-c2}
KN=${3:-K_parse}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
PASSES=${PASSES:-1234}
for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA" \
         "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU SQ_INSTS_SMEM" \
         "SQ_INSTS_VMEM SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_ACTIVE_INST_MISC SQ_IFETCH SQ_ACTIVE_INST_FLAT SQ_INSTS_BRANCH SQ_INSTS_VALU_INT32" \
         "SQ_ACTIVE_INST_VALU2 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_THREAD_CYCLES_VALU SQ_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_LDS_ATOMIC SQ_INSTS_VALU_IOPS"; do
  i=$((i+1))
  case $PASSES in *$i*) ;; *) continue ;; esac
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $P -d $OUT/p$i -o run --output-format csv -- \
    python3 $R/bench.py --config $CFG --steps 2 --warmup 1 --kernel-reps 2 --no-cpu-baseline --no-e2e --hbm-config "" > $OUT/p$i.log 2>&1 \
    || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 $R/scripts/pmcsum.py $OUT $KN | tee $OUT/summary.txt
