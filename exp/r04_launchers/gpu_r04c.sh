#!/bin/bash
set -o pipefail
# K_parse variants: timing (c2 all, c3 some), instruction counters, variant parity, then the product suite
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out; cd $R
V2="exp/v/base.so exp/v/v4a.so exp/v/v4b.so exp/v/v4c.so exp/v/v4d.so exp/v/v4e.so exp/v/v4f.so exp/v/v4g.so"
V3="exp/v/base.so exp/v/v4e.so exp/v/v4f.so exp/v/v4g.so"
echo "== c2" | tee -a gpurun_out/kp.txt
KEXP_CFG=c2 timeout -k 10 400 python -u scripts/kparse_only.py $V2 2>&1 | cut -c1-150 | tee -a gpurun_out/kp.txt || exit 1
echo "== c3" | tee -a gpurun_out/kp.txt
KEXP_CFG=c3 timeout -k 10 300 python -u scripts/kparse_only.py $V3 2>&1 | cut -c1-150 | tee -a gpurun_out/kp.txt || exit 1
for v in exp/v/base.so exp/v/v4e.so exp/v/v4g.so; do
  bash scripts/pmc_variant.sh pmc_$(basename $v .so) c2 $v > /dev/null || exit 1
  echo "== pmc $v"; grep -E "INSTS_VALU|INSTS_SALU|INSTS_LDS|WAVE_CYCLES|WAIT_ANY|WAIT_INST" gpurun_out/pmc_$(basename $v .so)/summary.txt
done 2>&1 | tee -a gpurun_out/kp.txt
MPC_TEST_LIB=exp/v/v4g.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_depth.py -x -q --timeout 300 --timeout-method thread > gpurun_out/tv.log 2>&1
rc=$?; echo "parity v4g:"; tail -2 gpurun_out/tv.log; [ $rc -eq 0 ] || { grep -E "^E |Error|FAILED" gpurun_out/tv.log | head -20; exit $rc; }
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t.log 2>&1
rc=$?; echo "product suite:"; tail -2 gpurun_out/t.log; [ $rc -eq 0 ] || { grep -E "^E |Error|FAILED" gpurun_out/t.log | head -20; exit $rc; }
timeout -k 10 300 python -u bench.py --hbm-config c3 > gpurun_out/b.log 2>&1 || { tail -20 gpurun_out/b.log; exit 1; }
grep -o '"value": [0-9.e+]*\|"ms_per_step": [0-9.]*\|"single_batch_ms_per_step": [0-9.]*\|"mean_launch_us": [0-9.]*' gpurun_out/b.log | head -8
timeout -k 10 200 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29541 \
  exp/dist_overhead.py c2 2>&1 | grep -v "^\[W\|Warning" | tee gpurun_out/dist_overhead.txt || exit 1
