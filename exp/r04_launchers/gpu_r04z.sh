#!/bin/bash
set -o pipefail
# tokenizer prototype v3b (units stored straight from the rounds): occupancy
# cap x wave count (one resident round of waves vs a tail round)
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out; cd $R
for wv in ${TOK_SWEEP:-4:6144 8:8192 4:12288}; do
  set -- ${wv/:/ }
  timeout -k 10 300 python3 -u exp/tok/run_tok.py --lib exp/tok/libtok_w$1.so --waves $2 --check c1,c2,c4 c1 c2 c4 c3 c5 > gpurun_out/tok_w$1_$2.txt 2>&1 || { tail -5 gpurun_out/tok_w$1_$2.txt; exit 1; }
  grep '^{' gpurun_out/tok_w$1_$2.txt | WAVES=$2 python3 -c "
import sys, json, os
for l in sys.stdin:
    r = json.loads(l)
    print('waves %s %s %s %8.1f us %6.1f GB/s check %s' % (os.environ['WAVES'], r['lib'], r['config'], r['median_us'], r['GB_per_s'], r.get('check', '-')))"
done
