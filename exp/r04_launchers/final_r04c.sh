#!/bin/bash
set -o pipefail
# C2 with 3 batches in flight (the new default): the in-flight GPU tests, the
# default bench line and the rocprofv3 kernel stats of that same command
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v -k "in_flight or nccl" --timeout 200 --timeout-method thread > gpurun_out/f4c_t.log 2>&1
rc=$?; grep -E "passed|failed|error" gpurun_out/f4c_t.log | tail -2; [ $rc -eq 0 ] || { grep -E "FAILED|^E " gpurun_out/f4c_t.log | head -30; exit $rc; }
timeout -k 10 400 python3 -u bench.py > gpurun_out/f4c_c2.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/f4c_c2.log; exit 1; }
grep '^{' gpurun_out/f4c_c2.log | tail -1 > gpurun_out/f4c_c2_bench.json; cut -c1-300 gpurun_out/f4c_c2_bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/f4c_c2_bench_ks -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-e2e > $R/gpurun_out/f4c_c2_bench_ks.log 2>&1 || { echo "rocprof bench failed"; tail -5 $R/gpurun_out/f4c_c2_bench_ks.log; exit 1; }
python3 $R/scripts/kstats.py $R/gpurun_out/f4c_c2_bench_ks 14
grep '^{' $R/gpurun_out/f4c_c2_bench_ks.log | tail -1 | cut -c1-300
