R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 200 python3 -u exp/overlap.py c2 2 3 > gpurun_out/ovg.txt 2>&1 || exit 1
MPC_PARSE_GEOMETRY=1,1024,16 timeout -k 10 200 python3 -u exp/overlap.py c2 1 2 3 >> gpurun_out/ovg.txt 2>&1 || exit 1
MPC_PARSE_GEOMETRY=1,512,16 timeout -k 10 200 python3 -u exp/overlap.py c2 1 2 3 >> gpurun_out/ovg.txt 2>&1 || exit 1
