#!/usr/bin/env python3
"""Per-kernel timing (HIP events, mpc_profile_kernel) of library variants on one config.
  python3 scripts/kexp.py lib1.so [lib2.so ...]   (each variant in a fresh subprocess)"""
import json, os, subprocess, sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import importlib, json, os, sys, time
import numpy as np, torch
sys.path.insert(0, %r)
pkg = importlib.import_module("minion-plasmid-consensus_amd")
eng = pkg.engine
eng.set_library(os.environ["KEXP_LIB"])  # variant build under test (experiments only)
cfg = os.environ.get("KEXP_CFG", "c2")
n, reads, prof, seed, anti = {"c2": (2686, 100000, "default", 2, True), "c4": (10000, 100000, "indel", 4, True),
                              "c3": (10000, 125000, "default", 3, False)}[cfg]
syn = pkg.synth.Synth(n=n, n_reads=reads, profile=prof, seed=seed, antisense=anti)
samples = [syn.sample(s) for s in range(2 if anti else 1)]
r = eng.Runner(samples)
for _ in range(3): r.step(0.1, 5.0)
r.check(); torch.cuda.synchronize()
out = {}
st = torch.cuda.current_stream()
for name, k in (("parse", eng.K_PARSE), ("left", eng.K_LEFT), ("ins", eng.K_INS), ("flank", eng.K_FLANK)):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(10)]
    for a, b in ev:
        if k == eng.K_INS:  # K_ins consumes the run tallies: refill them first (untimed)
            r.plan.profile_kernel(eng.K_LEFT)
        a.record(st); r.plan.profile_kernel(k); b.record(st)
    torch.cuda.synchronize()
    out[name] = float(np.median([a.elapsed_time(b) for a, b in ev])) * 1e3
st = r.plan.status()
out["status"] = [int(x) for x in st]
t0 = time.perf_counter()
for _ in range(20): r.step(0.1, 5.0)
torch.cuda.synchronize()
out["step"] = (time.perf_counter() - t0) / 20 * 1e6
r.step(0.1, 5.0); r.check()
print("KEXP", json.dumps(out))
''' % REPO
for lib in sys.argv[1:]:
    env = dict(os.environ, KEXP_LIB=os.path.abspath(lib))
    p = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
    line = [l for l in p.stdout.splitlines() if l.startswith("KEXP")]
    print(os.path.basename(lib), line[0][5:] if line else ("FAILED rc=%d %s" % (p.returncode, p.stderr[-800:])), flush=True)
