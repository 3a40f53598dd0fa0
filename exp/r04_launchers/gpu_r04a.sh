#!/bin/bash
set -o pipefail
# Round-4 GPU check: parity suite (incl. the RCCL world-1 test), default bench,
# and bench.py's distributed branch under torchrun at WORLD_SIZE=1 (RCCL).
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/t.log 2>&1
rc=$?
tail -3 gpurun_out/t.log
[ $rc -eq 0 ] || { grep -E "^E |Error|FAILED" gpurun_out/t.log | head -30; exit $rc; }
timeout -k 10 400 python -u bench.py > gpurun_out/b.log 2>&1 || { tail -20 gpurun_out/b.log; exit 1; }
grep metric gpurun_out/b.log | cut -c1-600
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --dist --steps 10 --warmup 3 --no-cpu-baseline --no-e2e --hbm-config '' > gpurun_out/bd.log 2>&1 || { tail -20 gpurun_out/bd.log; exit 1; }
grep metric gpurun_out/bd.log | cut -c1-400
