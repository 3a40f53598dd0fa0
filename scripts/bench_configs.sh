#!/bin/bash
# One bench line per config (N=1, no CPU baseline): bash scripts/bench_configs.sh c1 c3 c4 c5
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for c in "$@"; do
  timeout -k 10 300 python3 bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_$c.log 2>&1 || { echo "$c failed"; tail -5 gpurun_out/bench_$c.log; exit 1; }
  python3 - "$c" gpurun_out/bench_$c.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
print(sys.argv[1], "%.3e b/s" % d["value"], "%.1f us/step" % (1e3 * d["ms_per_step"]),
      "parse %.1f us" % d["roofline"]["mean_launch_us"], "frac %.4f" % d["roofline"]["frac"],
      "cs %d MB" % (d["config"]["cs_bytes_per_gpu"] >> 20))
PY
done
