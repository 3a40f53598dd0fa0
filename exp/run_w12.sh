R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
echo "== default" >> gpurun_out/w12.txt
timeout -k 10 200 python3 -u exp/overlap.py c2 1 2 3 >> gpurun_out/w12.txt 2>&1 || exit 1
for g in 1,2048,12 2,2048,12 1,2048,8; do
  echo "== $g" >> gpurun_out/w12.txt
  MPC_PARSE_GEOMETRY=$g timeout -k 10 200 python3 -u exp/overlap.py c2 1 2 3 >> gpurun_out/w12.txt 2>&1 || exit 1
done
for g in default 3,2048,12; do
  echo "== c3 $g" >> gpurun_out/w12.txt
  if [ $g = default ]; then timeout -k 10 300 python3 -u exp/overlap.py c3 2 >> gpurun_out/w12.txt 2>&1 || exit 1
  else MPC_PARSE_GEOMETRY=$g timeout -k 10 300 python3 -u exp/overlap.py c3 1 2 >> gpurun_out/w12.txt 2>&1 || exit 1; fi
done
