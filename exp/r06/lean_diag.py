#!/usr/bin/env python3
"""Windows of K_parse classified lean (diagnostic build exp/v/leandiag.so counts
all windows in status[6] and the others in status[7]).
  python3 exp/r06/lean_diag.py exp/v/leandiag.so c2 c3 ..."""
import importlib
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
pkg = importlib.import_module("minion-plasmid-consensus_amd")
eng = pkg.engine
eng.set_library(os.path.abspath(sys.argv[1]))
import bench  # noqa: E402
import torch  # noqa: E402

for cfg in sys.argv[2:]:
    samples, _ = bench.shard_samples(pkg, cfg, 0, 1)
    plan = eng.Plan(eng.Batch(samples))
    plan.phase("parse")
    torch.cuda.synchronize()
    st = [int(x) for x in plan.status()]
    print(cfg, "windows", st[6], "not lean", st[7], "status", st[:6], flush=True)
