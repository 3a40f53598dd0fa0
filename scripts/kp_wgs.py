#!/usr/bin/env python3
"""Parse phase of ONE library built with -DMPC_TUNING_OVERRIDES at several
parse-grid sizes (MPC_PARSE_WGS, read at plan creation), round-robin, HIP
events, median per size.
  KEXP_CFG=c3 python3 scripts/kp_wgs.py exp/v/tune.so 256 512 1024"""
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

cfg = os.environ.get("KEXP_CFG", "c3")
rounds, reps = int(os.environ.get("KEXP_ROUNDS", "3")), int(os.environ.get("KEXP_REPS", "10"))
eng.set_library(os.path.abspath(sys.argv[1]))
sizes = [int(x) for x in sys.argv[2:]]
samples, _ = bench.shard_samples(pkg, cfg, 0, 1)
batch = eng.Batch(samples)
st = torch.cuda.current_stream()
times = {w: [] for w in sizes}
for r in range(rounds):
    for w in sizes:
        os.environ["MPC_PARSE_WGS"] = str(w)
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
        times[w].append(float(np.median([a.elapsed_time(b) for a, b in ev])) * 1e3)
        if r == 0:
            info = plan.info()
            print("  wgs %d: tally_mode %d window %d waves %d workgroups %d overrides %d flags %d" % (
                w, info["tally_mode"], info["parse_window"], info["parse_waves"], info["parse_workgroups"],
                info["overrides"], int(plan.status()[0])), flush=True)
        del plan
for w in sizes:
    print("%s wgs %d parse %.1f us (rounds: %s)" % (cfg, w, float(np.median(times[w])), " ".join("%.1f" % x for x in times[w])), flush=True)
