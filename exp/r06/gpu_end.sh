#!/bin/bash
# round 6 end: smoke, GPU suite, bench lines + single-batch kernel stats per config, and the default C2 command under rocprofv3
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r6z}
cd $R && mkdir -p gpurun_out
bash exp/r06/gpu_final.sh $TAG || exit 1
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out/${TAG}_c2default
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${TAG}_c2default -o run --output-format csv -- python3 $R/bench.py > $R/gpurun_out/${TAG}_c2default/bench.log 2>&1 || { echo "default bench under rocprof failed"; tail -5 $R/gpurun_out/${TAG}_c2default/bench.log; exit 1; }
grep '^{' $R/gpurun_out/${TAG}_c2default/bench.log | tail -1 > $R/gpurun_out/${TAG}_c2default/bench.json
python3 $R/scripts/kstats.py $R/gpurun_out/${TAG}_c2default 14
