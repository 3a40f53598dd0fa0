#!/bin/bash
set -o pipefail
# SQ counters of the prototype tokenizer at C3 (two passes of <= 8 SQ counters)
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/tokpmc; cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_ANY SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set -d $R/gpurun_out/tokpmc/p$i -o run --output-format csv -- \
    python3 $R/exp/tok/run_tok.py --check none --reps 2 c3 > $R/gpurun_out/tokpmc/p$i.log 2>&1 || { tail -5 $R/gpurun_out/tokpmc/p$i.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections, os
R=os.environ.get("GRAFT_REPO_ROOT", ".")
acc=collections.defaultdict(list)
for f in glob.glob(R+"/gpurun_out/tokpmc/p*/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        if "K_tok" in row.get("Kernel_Name",""):
            acc[row["Counter_Name"]].append(float(row["Counter_Value"]))
for k,v in sorted(acc.items()):
    print("%-24s %16.1f (n=%d)" % (k, sum(v)/len(v)*0 + sum(v)/ (len(v)/max(1,len(set(v)) and 1)), len(v)))
PY
