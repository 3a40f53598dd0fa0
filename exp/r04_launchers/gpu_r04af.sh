#!/bin/bash
set -o pipefail
# N>1 bench path rehearsal with the new defaults (C2: 3 pipelines, 3 process groups per rank;
# C1: 4): 2 and 4 ranks sharing cuda:0 over gloo
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for v in "2 c2" "4 c2" "2 c1"; do
  set -- $v
  bash scripts/dist_rehearsal.sh $1 $2 > /dev/null || { tail -20 gpurun_out/dist_$1.log; exit 1; }
  grep '^{' gpurun_out/dist_$1.log | tail -1 | python3 -c "
import sys, json
r = json.loads(sys.stdin.read())
print('ranks %d %s: ms_per_step %.3f value %.4g in_flight %d group %s' % (r['n_gpus'], r['config']['workload'][:3], r['ms_per_step'], r['value'], r['config']['batches_in_flight'], r['config']['process_group']))"
  cp gpurun_out/dist_$1.log gpurun_out/dist_$1_$2.log
done
