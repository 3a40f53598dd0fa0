#!/bin/bash
# Build experiment variants of libmpc.so into build/variants/ (travel to the GPU box; git-ignored).
R=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p $R/build/variants
for v in "$@"; do
  name=${v%%=*}; flags=${v#*=}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -I $R/include -I $R/minion-plasmid-consensus_amd/csrc \
    $flags -o $R/build/variants/$name.so $R/minion-plasmid-consensus_amd/csrc/mpc_kernels.hip &
done
wait
ls -la $R/build/variants
