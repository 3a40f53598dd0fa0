cd ${GRAFT_REPO_ROOT:-$(pwd)} && mkdir -p gpurun_out
for c in c2 c3 c5; do KEXP_CFG=$c timeout -k 10 300 python3 -u scripts/kparse_only.py exp/v/g256u1.so exp/v/pf.so exp/v/g256u1.so exp/v/pf.so >> gpurun_out/pf.txt 2>&1 || exit 1; done
bash exp/var_kstats.sh nf c3 exp/v/g256u1.so exp/v/noflush.so >> gpurun_out/pf.txt 2>&1
