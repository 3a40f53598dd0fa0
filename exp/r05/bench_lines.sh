#!/bin/bash
# bench lines per config (+ rocprofv3 kernel stats of the default C2 command)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for c in "$@"; do
  timeout -k 10 600 python3 -u bench.py --config $c > gpurun_out/bench_$c.json.log 2>&1 || { echo "bench $c failed"; tail -20 gpurun_out/bench_$c.json.log; exit 1; }
  python3 - $c gpurun_out/bench_$c.json.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
print(sys.argv[1], "%.3e b/s" % d["value"], "%.1f us/step" % (1e3 * d["ms_per_step"]), "single %.1f" % (1e3 * d["single_batch_ms_per_step"]),
      "parse %.1f us" % d["roofline"]["mean_launch_us"], "frac %.4f" % d["roofline"]["frac"], "traffic %s" % d["roofline"]["traffic"],
      "hbm", (d.get("roofline_hbm") or {}).get("frac"), "e2e", (d.get("e2e") or {}).get("wall_s"))
PY
done
