#!/usr/bin/env python3
"""Time ONE pipeline kernel of library variants (experiments): one full step,
then the kernel alone re-launched through mpc_profile_kernel (HIP events,
median of 15).  Re-launches add to stale tallies: timing only.
  KEXP_CFG=c1..c5 [KEXP_WORLD=N] KEXP_KERNEL=parse|left|flank|ins|rsort python3 scripts/kernel_only.py lib1.so [lib2.so ...]"""
import os, subprocess, sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import importlib, os, sys
import numpy as np, torch
sys.path.insert(0, %r)
pkg = importlib.import_module("minion-plasmid-consensus_amd")
eng = pkg.engine
eng.set_library(os.environ["KEXP_LIB"])  # variant build under test (experiments only)
import bench
# KEXP_WORLD=N: rank 0's read slice of an N-GPU run, as one single-GPU batch
samples, _ = bench.shard_samples(pkg, os.environ.get("KEXP_CFG", "c2"), 0, int(os.environ.get("KEXP_WORLD", "1")))
which = {"parse": eng.K_PARSE, "left": eng.K_LEFT, "flank": eng.K_FLANK, "ins": eng.K_INS, "rsort": eng.K_RSORT}[os.environ.get("KEXP_KERNEL", "flank")]
runner = eng.Runner(samples)
runner.step(0.1, 5.0)
st = torch.cuda.current_stream()
for _ in range(3): runner.plan.profile_kernel(which)
torch.cuda.synchronize()
ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(15)]
for a, b in ev:
    a.record(st); runner.plan.profile_kernel(which); b.record(st)
torch.cuda.synchronize()
print("KT %%.1f" %% float(np.median([a.elapsed_time(b) for a, b in ev]) * 1e3))
''' % REPO
for lib in sys.argv[1:]:
    env = dict(os.environ, KEXP_LIB=os.path.abspath(lib))
    p = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
    line = [l for l in p.stdout.splitlines() if l.startswith("KT")]
    print(os.path.basename(lib), line[0][3:] if line else ("FAILED rc=%d %s" % (p.returncode, p.stderr[-800:])), flush=True)
