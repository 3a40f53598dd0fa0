#!/bin/bash
set -o pipefail
# smoke, the GPU suite, the default bench line and the rocprofv3 kernel stats
# of the same command; then the distributed step eager vs HIP-graph replay
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/f4_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/f4_smoke.log; exit 1; }
tail -1 gpurun_out/f4_smoke.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/f4_t.log 2>&1
rc=$?; grep -E "passed|failed|error" gpurun_out/f4_t.log | tail -2; [ $rc -eq 0 ] || { grep -E "FAILED|^E " gpurun_out/f4_t.log | head -30; exit $rc; }
timeout -k 10 400 python3 -u bench.py > gpurun_out/f4_c2.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/f4_c2.log; exit 1; }
grep '^{' gpurun_out/f4_c2.log | tail -1 > gpurun_out/f4_c2_bench.json; cut -c1-300 gpurun_out/f4_c2_bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/f4_c2_bench_ks -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-e2e > $R/gpurun_out/f4_c2_bench_ks.log 2>&1 || { echo "rocprof bench failed"; tail -5 $R/gpurun_out/f4_c2_bench_ks.log; exit 1; }
python3 $R/scripts/kstats.py $R/gpurun_out/f4_c2_bench_ks 14
cd $R
timeout -k 10 200 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29542 \
  exp/dist_graph.py c2 2>&1 | grep -v "^\[W\|Warning" | tee gpurun_out/dist_graph.txt
