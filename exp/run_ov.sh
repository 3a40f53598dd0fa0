R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python3 -u exp/overlap.py c2 1 2 3 > gpurun_out/ov.txt 2>&1 || exit 1
timeout -k 10 300 python3 -u exp/overlap.py c3 1 2 >> gpurun_out/ov.txt 2>&1 || exit 1
bash scripts/pmc_traffic.sh r03tr c2 c3 c4 > gpurun_out/r03tr.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r03def -o run --output-format csv -- python3 $R/bench.py > $R/gpurun_out/r03def_bench.log 2>&1
