R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for w in 256 128 64; do
  echo "== c1 wgs $w" >> gpurun_out/wgs.txt
  MPC_PARSE_WGS=$w timeout -k 10 200 python3 -u exp/overlap.py c1 1 2 >> gpurun_out/wgs.txt 2>&1 || exit 1
done
