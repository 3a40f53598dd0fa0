#!/bin/bash
set -o pipefail
# prototype tokenizer (pass 1 of a split parse): timing at C1-C5, unit stream
# checked against exp/tok/tok_ref.c at C1 / C2 / C4
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out; cd $R
timeout -k 10 400 python3 -u exp/tok/run_tok.py --check c1,c2,c4 c1 c2 c4 c3 c5 > gpurun_out/tok_proto.txt 2>&1
rc=$?; cat gpurun_out/tok_proto.txt | grep -v amdgpu.ids; exit $rc
