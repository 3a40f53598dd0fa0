#!/bin/bash
# Rehearse the N>1 bench path on a one-GPU box: N ranks share cuda:0 and exchange
# over gloo (RCCL needs one GPU per rank).  bash scripts/dist_rehearsal.sh [N] [config]
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
N=${1:-2}
CFG=${2:-c2}
MPC_DIST_BACKEND=gloo timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus $N --config $CFG --steps 5 --warmup 2 \
  > gpurun_out/dist_$N.log 2>&1
rc=$?
tail -4 gpurun_out/dist_$N.log
exit $rc
