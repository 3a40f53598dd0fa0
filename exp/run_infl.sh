R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-e2e > gpurun_out/infl_c2.log 2>&1 || { tail -20 gpurun_out/infl_c2.log; exit 1; }
timeout -k 10 300 python3 -u bench.py --inflight 1 --no-cpu-baseline --no-e2e --hbm-config "" > gpurun_out/infl1_c2.log 2>&1 || exit 1
bash scripts/dist_rehearsal.sh 2 c2 || exit 1
bash scripts/dist_rehearsal.sh 2 c3
