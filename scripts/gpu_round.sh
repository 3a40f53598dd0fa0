#!/bin/bash
# GPU round trip: smoke, all -m gpu tests, then bench lines.  bash scripts/gpu_round.sh [configs...]
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed rc=$?"; tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1
rc=$?
grep -E "passed|failed|error" gpurun_out/t.log | tail -3
[ $rc -eq 0 ] || { grep -E "FAILED|^E " gpurun_out/t.log | head -30; exit $rc; }
for c in "$@"; do
  timeout -k 10 400 python -u bench.py --config $c > gpurun_out/bench_$c.log 2>&1 || { echo "bench $c failed"; tail -20 gpurun_out/bench_$c.log; exit 1; }
  python3 - $c gpurun_out/bench_$c.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
print(sys.argv[1], "%.3e b/s" % d["value"], "%.1f us/step" % (1e3 * d["ms_per_step"]),
      "parse %.1f us" % d["roofline"]["mean_launch_us"], "frac %.4f" % d["roofline"]["frac"])
PY
done
