#!/usr/bin/env python3
"""MPC_ST_SPEC after one parse per config (1: the speculative pass met a unit it
does not decode and the exact pass redid the parse).
  python3 exp/r06/spec_diag.py c1 c2 ..."""
import importlib
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
pkg = importlib.import_module("minion-plasmid-consensus_amd")
eng = pkg.engine
import bench  # noqa: E402
import torch  # noqa: E402

for cfg in sys.argv[1:]:
    samples, _ = bench.shard_samples(pkg, cfg, 0, 1)
    plan = eng.Plan(eng.Batch(samples))
    plan.phase("parse")
    torch.cuda.synchronize()
    st = [int(x) for x in plan.status()]
    print(cfg, "spec_failed", st[eng.MPC_ST_SPEC], "status", st, flush=True)
