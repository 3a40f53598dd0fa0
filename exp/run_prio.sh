R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for rep in 1 2; do
for v in noprio prio2 prio3; do
  echo "== $v" >> gpurun_out/prio.txt
  KEXP_LIB=exp/v/$v.so timeout -k 10 200 python3 -u exp/overlap.py c2 1 2 >> gpurun_out/prio.txt 2>&1 || exit 1
done
done
for v in noprio prio3; do
  echo "== c3 $v" >> gpurun_out/prio.txt
  KEXP_LIB=exp/v/$v.so timeout -k 10 300 python3 -u exp/overlap.py c3 2 >> gpurun_out/prio.txt 2>&1 || exit 1
done
