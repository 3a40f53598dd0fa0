#!/usr/bin/env python3
"""Run full steps of ONE library variant in-process (for rocprofv3 kernel stats):
  python3 exp/var_steps.py exp/v/a.so c2 [steps]"""
import importlib
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

pkg = importlib.import_module("minion-plasmid-consensus_amd")
eng = pkg.engine
eng.set_library(os.path.abspath(sys.argv[1]))  # variant build under test (experiments only)
import bench  # noqa: E402

samples, _ = bench.shard_samples(pkg, sys.argv[2], 0, 1)
runner = eng.Runner(samples)
for _ in range(int(sys.argv[3]) if len(sys.argv) > 3 else 10):
    runner.step(0.1, 5.0)
torch.cuda.synchronize()
runner.check()
print("ok", sys.argv[1], sys.argv[2])
