cd ${GRAFT_REPO_ROOT:-$(pwd)} && mkdir -p gpurun_out
for c in c2 c3; do KEXP_CFG=$c timeout -k 10 300 python3 -u scripts/kparse_only.py exp/v/base.so exp/v/notally.so exp/v/base.so exp/v/notally.so >> gpurun_out/nt.txt 2>&1 || exit 1; done
