#!/bin/bash
# bash exp/abl/build.sh <name> [-DMPC_ABL_...]: timing-only variant from exp/abl/abl.hip
R=$(cd "$(dirname "$0")/../.." && pwd)
N=$1; shift
mkdir -p $R/exp/v
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -I $R/include -I $R/minion-plasmid-consensus_amd/csrc \
  -o $R/exp/v/$N.so "$@" $R/exp/abl/abl.hip 2>&1 | grep -v "hip-link"
test -f $R/exp/v/$N.so
