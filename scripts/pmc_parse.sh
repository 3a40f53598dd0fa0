#!/bin/bash
# PMC passes for the dominant kernel (run on the GPU box from the repo root).
# Each pass is its own rocprofv3 run with --kernel-trace only (no other trace domains).
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-pmc}
CFG=${2:-c2}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for P in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
         "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM GRBM_GUI_ACTIVE" \
         "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_ATOMIC_sum TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $P -d $OUT/p$i -o run --output-format csv -- \
    python3 $R/bench.py --config $CFG --steps 3 --warmup 1 --kernel-reps 3 --no-cpu-baseline > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done
echo done
