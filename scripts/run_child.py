#!/usr/bin/env python3
"""Full pileup steps (every phase) of ONE library variant on one config, for
rocprofv3 kernel stats of experiment builds (ablation variants give wrong
results: no check).  KEXP_LIB=exp/v/x.so KEXP_CFG=c3 [KEXP_STEPS=10] python3 scripts/run_child.py"""
import importlib
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
pkg = importlib.import_module("minion-plasmid-consensus_amd")
eng = pkg.engine
if os.environ.get("KEXP_LIB"):
    eng.set_library(os.path.abspath(os.environ["KEXP_LIB"]))
import bench  # noqa: E402

samples, _ = bench.shard_samples(pkg, os.environ.get("KEXP_CFG", "c3"), 0, 1)
runner = eng.Runner(samples)
for _ in range(int(os.environ.get("KEXP_STEPS", "10"))):
    runner.step(0.1, 5.0)
torch.cuda.synchronize()
print("RUN ok", [int(x) for x in runner.plan.status()][:4], flush=True)
