#!/bin/bash
# bench.py line per (library variant, config): bash scripts/variant_bench.sh "c2 c4 c5" build/variants/*.so
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
cfgs=$1; shift
for lib in "$@"; do
  for c in $cfgs; do
    MPC_LIB=$R/$lib timeout -k 10 200 python3 bench.py --config $c --steps 5 --warmup 2 --kernel-reps 5 --no-cpu-baseline > gpurun_out/vb.log 2>&1 || { echo "$lib $c failed"; tail -5 gpurun_out/vb.log; exit 1; }
    python3 - "$lib" "$c" gpurun_out/vb.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[3]) if l.startswith("{")][-1])
print(sys.argv[1].split("/")[-1], sys.argv[2], "%.3e b/s" % d["value"], "%.1f us/step" % (1e3 * d["ms_per_step"]),
      "parse %.1f us" % d["roofline"]["mean_launch_us"], flush=True)
PY
  done
done
