R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for w in 256 224 192 160 128; do
  echo "== c2 wgs $w" >> gpurun_out/wgs2.txt
  MPC_PARSE_WGS=$w timeout -k 10 200 python3 -u exp/overlap.py c2 2 3 >> gpurun_out/wgs2.txt 2>&1 || exit 1
done
for w in 256 224 192; do
  echo "== c3 wgs $w" >> gpurun_out/wgs2.txt
  MPC_PARSE_WGS=$w timeout -k 10 300 python3 -u exp/overlap.py c3 2 >> gpurun_out/wgs2.txt 2>&1 || exit 1
done
