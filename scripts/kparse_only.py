#!/usr/bin/env python3
"""Time the parse phase ALONE (K_clear + K_parse, HIP events) of library
variants; later phases never run, so experiment builds that skip stores are
safe.   KEXP_CFG=c1..c5 (bench.py workloads) python3 scripts/kparse_only.py lib1.so [lib2.so ...]"""
import os, subprocess, sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import importlib, os, sys
import numpy as np, torch
sys.path.insert(0, %r)
pkg = importlib.import_module("minion-plasmid-consensus_amd")
eng = pkg.engine
eng.set_library(os.environ["KEXP_LIB"])  # variant build under test (experiments only)
cfg = os.environ.get("KEXP_CFG", "c2")
sys.path.insert(0, %r)
import bench
samples, _ = bench.shard_samples(pkg, cfg, 0, 1)
plan = eng.Plan(eng.Batch(samples))
st = torch.cuda.current_stream()
for _ in range(3): plan.phase("parse")
torch.cuda.synchronize()
ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(15)]
for a, b in ev:
    a.record(st); plan.phase("parse"); b.record(st)
torch.cuda.synchronize()
print("KP %%.1f" %% float(np.median([a.elapsed_time(b) for a, b in ev]) * 1e3), [int(x) for x in plan.status()][:4])
''' % (REPO, REPO)
for lib in sys.argv[1:]:
    env = dict(os.environ, KEXP_LIB=os.path.abspath(lib))
    p = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
    line = [l for l in p.stdout.splitlines() if l.startswith("KP")]
    print(os.path.basename(lib), line[0][3:] if line else ("FAILED rc=%d %s" % (p.returncode, p.stderr[-800:])), flush=True)
