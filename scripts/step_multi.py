#!/usr/bin/env python3
"""Full single-batch steps (mpc_run: parse -> consensus) of several library
variants on one config in ONE process, round-robin; HIP events, median per
variant; also the parse phase alone (K_clear + K_parse [+ K_subs]).
  KEXP_CFG=c4 [KEXP_ROUNDS=3] [KEXP_REPS=10] python3 scripts/step_multi.py a.so b.so ..."""
import importlib
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
pkg = importlib.import_module("minion-plasmid-consensus_amd")
eng = pkg.engine
import bench  # noqa: E402

cfg = os.environ.get("KEXP_CFG", "c2")
rounds = int(os.environ.get("KEXP_ROUNDS", "3"))
reps = int(os.environ.get("KEXP_REPS", "10"))
libs = [os.path.abspath(p) for p in sys.argv[1:]]
eng.LIB_PATH = libs[0]
eng.lib()
if os.environ.get("KEXP_SYNTH"):  # "n,reads": one synthetic sample of that shape instead of a bench config
    n_, r_ = (int(x) for x in os.environ["KEXP_SYNTH"].split(","))
    samples = [pkg.synth.Synth(n=n_, n_reads=r_, profile="default", seed=5, frac_partial=0.1).sample(0)]
    cfg = "synth%d_%d" % (n_, r_)
else:
    samples, _ = bench.shard_samples(pkg, cfg, 0, 1)
batch = eng.Batch(samples)
st = torch.cuda.current_stream()
times = {p: ([], []) for p in libs}


def timed(fn):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record(st)
        fn()
        b.record(st)
    torch.cuda.synchronize()
    return float(np.median([a.elapsed_time(b) for a, b in ev])) * 1e3


for r in range(rounds):
    for p in libs:
        eng._lib = None  # (experiments only) switch the variant
        eng.LIB_PATH = p
        plan = eng.Plan(batch)
        plan.run(0.1, 5.0)
        st_ = plan.status()
        if int(st_[eng.MPC_ST_FLAGS]) & eng.DE_CAPACITY:
            plan = eng.Plan(batch, int(st_[eng.MPC_ST_ROWS_NEEDED]) + 16)
        for _ in range(2):
            plan.run(0.1, 5.0)
        torch.cuda.synchronize()
        flags = int(plan.status()[eng.MPC_ST_FLAGS])
        times[p][0].append(timed(lambda: plan.run(0.1, 5.0)))
        times[p][1].append(timed(lambda: plan.phase("parse")))
        plan.run(0.1, 5.0)
        torch.cuda.synchronize()
        if r == 0:
            print("  %s: flags %d" % (os.path.basename(p), flags), flush=True)
        plan.h, h = None, plan.h
        eng._lib.mpc_plan_destroy(h)
        del plan
for p in libs:
    s, k = times[p]
    print("%s %s step %.1f us parse %.1f us (steps: %s)" % (cfg, os.path.basename(p), float(np.median(s)),
                                                             float(np.median(k)), " ".join("%.1f" % x for x in s)),
          flush=True)
