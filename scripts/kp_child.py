#!/usr/bin/env python3
"""Parse phase (K_clear + K_parse [+ K_subs]) of ONE library variant on one
config, HIP events: the child of scripts/kparse_only.py, also run directly
under rocprofv3 (counters per variant).
  KEXP_LIB=exp/v/x.so KEXP_CFG=c2 [KEXP_REPS=15] python3 scripts/kp_child.py"""
import importlib
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
pkg = importlib.import_module("minion-plasmid-consensus_amd")
eng = pkg.engine
if os.environ.get("KEXP_LIB"):
    eng.set_library(os.path.abspath(os.environ["KEXP_LIB"]))  # variant build under test (experiments only)
import bench  # noqa: E402

cfg = os.environ.get("KEXP_CFG", "c2")
reps = int(os.environ.get("KEXP_REPS", "15"))
samples, _ = bench.shard_samples(pkg, cfg, 0, 1)
plan = eng.Plan(eng.Batch(samples))
st = torch.cuda.current_stream()
for _ in range(3):
    plan.phase("parse")
torch.cuda.synchronize()
ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
for a, b in ev:
    a.record(st)
    plan.phase("parse")
    b.record(st)
torch.cuda.synchronize()
print("KP %.1f" % float(np.median([a.elapsed_time(b) for a, b in ev]) * 1e3), [int(x) for x in plan.status()][:4],
      plan.info(), flush=True)
