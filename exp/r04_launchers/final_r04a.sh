#!/bin/bash
set -o pipefail
# Round-4 final measurements, part 1: smoke, the GPU suite, the default bench
# line (C2, 2 batches in flight) and the rocprofv3 kernel stats of that same
# command, K_parse HBM traffic (PMC) at C2 and C3
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/f4_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/f4_smoke.log; exit 1; }
tail -1 gpurun_out/f4_smoke.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/f4_t.log 2>&1
rc=$?; grep -E "passed|failed|error" gpurun_out/f4_t.log | tail -2; [ $rc -eq 0 ] || { grep -E "FAILED|^E " gpurun_out/f4_t.log | head -30; exit $rc; }
timeout -k 10 400 python3 -u bench.py > gpurun_out/f4_c2.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/f4_c2.log; exit 1; }
grep '^{' gpurun_out/f4_c2.log | tail -1 > gpurun_out/f4_c2_bench.json; cut -c1-400 gpurun_out/f4_c2_bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/f4_c2_bench_ks -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-e2e > $R/gpurun_out/f4_c2_bench_ks.log 2>&1 || { echo "rocprof bench failed"; tail -5 $R/gpurun_out/f4_c2_bench_ks.log; exit 1; }
python3 $R/scripts/kstats.py $R/gpurun_out/f4_c2_bench_ks 14
grep '^{' $R/gpurun_out/f4_c2_bench_ks.log | tail -1 | cut -c1-300
cd $R && bash scripts/pmc_traffic.sh f4pmc c2 c3 || exit 1
cat gpurun_out/pmc_traffic_c2.json gpurun_out/pmc_traffic_c3.json
