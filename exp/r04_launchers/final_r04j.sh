#!/bin/bash
set -o pipefail
# rocprofv3 kernel stats with the final kernels: the default bench command (C2, 3 in flight)
# and the one-batch C2 command (whose K_parse mean is the bench line's roofline launch)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/f4j_c2_default -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-e2e > $R/gpurun_out/f4j_c2_default.log 2>&1 || { echo "rocprof default failed"; tail -5 $R/gpurun_out/f4j_c2_default.log; exit 1; }
python3 $R/scripts/kstats.py $R/gpurun_out/f4j_c2_default 6
grep '^{' $R/gpurun_out/f4j_c2_default.log | tail -1 | python3 -c "import sys, json; r = json.loads(sys.stdin.read()); print('default line: us/step %.1f, roofline K_parse %.1f us' % (r['ms_per_step'] * 1e3, r['roofline']['mean_launch_us']))"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/f4j_c2_single -o run --output-format csv -- python3 $R/bench.py --inflight 1 --no-cpu-baseline --no-e2e --hbm-config= > $R/gpurun_out/f4j_c2_single.log 2>&1 || { echo "rocprof single failed"; tail -5 $R/gpurun_out/f4j_c2_single.log; exit 1; }
python3 $R/scripts/kstats.py $R/gpurun_out/f4j_c2_single 6
grep '^{' $R/gpurun_out/f4j_c2_single.log | tail -1 | python3 -c "import sys, json; r = json.loads(sys.stdin.read()); print('one-batch line: us/step %.1f, roofline K_parse %.1f us' % (r['ms_per_step'] * 1e3, r['roofline']['mean_launch_us']))"
