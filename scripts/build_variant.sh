#!/bin/bash
# Build an experiment variant of libmpc.so into exp/v/<name>.so from the current
# source with extra -D switches:  bash scripts/build_variant.sh <name> [-DFOO ...]
R=$(cd "$(dirname "$0")/.." && pwd)
N=$1; shift
mkdir -p $R/exp/v
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -I $R/include -I $R/minion-plasmid-consensus_amd/csrc \
  -o $R/exp/v/$N.so "$@" $R/minion-plasmid-consensus_amd/csrc/mpc_kernels.hip 2>&1 | grep -v "hip-link" 
test -f $R/exp/v/$N.so
