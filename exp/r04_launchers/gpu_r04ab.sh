#!/bin/bash
set -o pipefail
# the distributed bench path (RCCL, world size 1 via torch.distributed.run) with the
# new C2 default of 3 pipelines in flight: eager and graph replay
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out; cd $R
for g in "" "--graph"; do
  timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 \
    bench.py --gpus 1 --dist $g --no-cpu-baseline --no-e2e --hbm-config '' > gpurun_out/dist3$g.log 2>&1 || { tail -20 gpurun_out/dist3$g.log; exit 1; }
  grep '^{' gpurun_out/dist3$g.log | tail -1 | python3 -c "
import sys, json
r = json.loads(sys.stdin.read())
print('dist %s: ms_per_step %.4f value %.4g in_flight %d graph %s group %s' % ('$g' or 'eager', r['ms_per_step'], r['value'], r['config']['batches_in_flight'], r['config']['graph'], r['config']['process_group']))"
done
