#!/bin/bash
set -o pipefail
# K_parse variants: timing (c2, c3), instruction counters, variant parity
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out; cd $R
V="${VARIANTS:-exp/v/base.so exp/v/v4a.so exp/v/v4b.so exp/v/v4c.so exp/v/v4d.so exp/v/v4e.so exp/v/v4f.so exp/v/v4g.so}"
P="${PARITY:-exp/v/v4f.so exp/v/v4g.so}"
for cfg in c2 c3; do
  KEXP_CFG=$cfg timeout -k 10 400 python -u scripts/kparse_only.py $V 2>&1 | cut -c1-150 | tee -a gpurun_out/kp.txt || exit 1
done
for v in $V; do
  bash scripts/pmc_variant.sh pmc_$(basename $v .so) c2 $v > /dev/null || exit 1
  echo "== $v"; grep -E "INSTS_VALU|INSTS_SALU|INSTS_LDS|WAVE_CYCLES|WAIT_ANY|WAIT_INST" gpurun_out/pmc_$(basename $v .so)/summary.txt
done 2>&1 | tee -a gpurun_out/kp.txt
for p in $P; do
  MPC_TEST_LIB=$p timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_depth.py -x -q --timeout 400 --timeout-method thread > gpurun_out/tv.log 2>&1
  rc=$?; echo "parity $p:"; tail -2 gpurun_out/tv.log; [ $rc -eq 0 ] || { grep -E "^E |Error|FAILED" gpurun_out/tv.log | head -20; exit $rc; }
done
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29541 \
  exp/dist_overhead.py c2 2>&1 | grep -v "^\[W\|Warning" | tee gpurun_out/dist_overhead.txt || exit 1
