#!/usr/bin/env python3
"""Full-step timing (mpc_run, HIP events, median of 20) of exp/v variant libraries.
  KEXP_CFG=c2 python3 exp/step_time.py exp/v/a.so exp/v/b.so ..."""
import os, subprocess, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import importlib, os, sys
import numpy as np, torch
sys.path.insert(0, %r)
pkg = importlib.import_module("minion-plasmid-consensus_amd")
eng = pkg.engine
eng.set_library(os.environ["KEXP_LIB"])
import bench
samples, _ = bench.shard_samples(pkg, os.environ.get("KEXP_CFG", "c2"), 0, 1)
runner = eng.Runner(samples)
runner.step(0.1, 5.0)
st = torch.cuda.current_stream()
for _ in range(3): runner.step(0.1, 5.0)
torch.cuda.synchronize()
ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(20)]
for a, b in ev:
    a.record(st); runner.step(0.1, 5.0); b.record(st)
torch.cuda.synchronize()
runner.check()
print("ST %%.1f" %% float(np.median([a.elapsed_time(b) for a, b in ev]) * 1e3))
''' % REPO
for lib in sys.argv[1:]:
    env = dict(os.environ, KEXP_LIB=os.path.abspath(lib))
    p = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
    line = [l for l in p.stdout.splitlines() if l.startswith("ST")]
    print(os.path.basename(lib), line[0][3:] if line else ("FAILED rc=%d %s" % (p.returncode, p.stderr[-800:])), flush=True)
