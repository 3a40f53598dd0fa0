#!/usr/bin/env python3
"""Parse phase (K_clear + K_parse [+ K_subs]) of several library variants on
one config in ONE process (the samples are generated once), round-robin so
that drift hits every variant alike; HIP events, median per variant.
  KEXP_CFG=c2 [KEXP_ROUNDS=3] [KEXP_REPS=10] python3 scripts/kp_multi.py a.so b.so ..."""
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
eng.lib()  # the first variant loads the HIP runtime the same way the product does
samples, _ = bench.shard_samples(pkg, cfg, 0, 1)
batch = eng.Batch(samples)
st = torch.cuda.current_stream()
times = {p: [] for p in libs}
for r in range(rounds):
    for p in libs:
        eng._lib = None  # (experiments only) switch the variant: plans of the previous one are gone
        eng.LIB_PATH = p
        plan = eng.Plan(batch)
        for _ in range(2):
            plan.phase("parse")
        torch.cuda.synchronize()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
        for a, b in ev:
            a.record(st)
            plan.phase("parse")
            b.record(st)
        torch.cuda.synchronize()
        times[p].append(float(np.median([a.elapsed_time(b) for a, b in ev])) * 1e3)
        if r == 0:
            info = plan.info()
            print("  %s: tally_mode %d window %d lds %d wg %d flags %d" % (
                os.path.basename(p), info["tally_mode"], info["parse_window"], info["parse_lds_bytes"],
                info["parse_workgroups"], int(plan.status()[0])), flush=True)
        plan.h, h = None, plan.h
        eng._lib.mpc_plan_destroy(h)
        del plan
for p in libs:
    t = times[p]
    print("%s %s %.1f us (rounds: %s)" % (cfg, os.path.basename(p), float(np.median(t)), " ".join("%.1f" % x for x in t)),
          flush=True)
