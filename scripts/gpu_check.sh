#!/bin/bash
# GPU round trip: parity tests, bench line, kernel stats.  bash scripts/gpu_check.sh [bench args...]
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/t.log 2>&1
rc=$?
tail -3 gpurun_out/t.log
[ $rc -eq 0 ] || { grep -E "^E |Error" gpurun_out/t.log | head -20; exit $rc; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 "$@" > gpurun_out/b.log 2>&1 || { tail -20 gpurun_out/b.log; exit 1; }
grep metric gpurun_out/b.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $R/gpurun_out/p.log 2>&1 || { tail -20 $R/gpurun_out/p.log; exit 1; }
python3 $R/scripts/kstats.py $R/gpurun_out/prof 14
