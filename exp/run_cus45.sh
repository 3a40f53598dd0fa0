R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for c in c4 c5; do
  for n in 256 224 192 160; do
    echo "== $c parse_cus $n" >> gpurun_out/cus45.txt
    PARSE_CUS=$n timeout -k 10 240 python3 -u exp/overlap.py $c 2 >> gpurun_out/cus45.txt 2>&1 || exit 1
  done
done
