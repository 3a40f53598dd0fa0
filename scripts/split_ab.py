#!/usr/bin/env python3
"""Parse phase (K_clear + K_parse) with the work split by cs bytes vs by read
count, interleaved in one process (HIP events, median of 15).
  python3 scripts/split_ab.py c2 c3 c4"""
import importlib
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
pkg = importlib.import_module("minion-plasmid-consensus_amd")
eng = pkg.engine
bench = importlib.import_module("bench")


def timed(plan, reps=15):
    st = torch.cuda.current_stream()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record(st)
        plan.phase("parse")
        b.record(st)
    torch.cuda.synchronize()
    return float(np.median([a.elapsed_time(b) for a, b in ev]) * 1e3)


for cfg in sys.argv[1:] or ["c2"]:
    samples, _ = bench.shard_samples(pkg, cfg, 0, 1)
    plans = {k: eng.Plan(eng.Batch(samples, balance_bytes=k == "bytes")) for k in ("count", "bytes")}
    for p in plans.values():
        for _ in range(3):
            p.phase("parse")
    torch.cuda.synchronize()
    res = {k: [] for k in plans}
    for _ in range(3):
        for k, p in plans.items():
            res[k].append(timed(p))
    print(cfg, {k: round(float(np.median(v)), 1) for k, v in res.items()}, flush=True)
    del plans
    torch.cuda.empty_cache()
