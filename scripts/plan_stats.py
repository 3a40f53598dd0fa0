#!/usr/bin/env python3
"""One step per bench config; prints the plan's status words (rows needed,
mixed RIGHT events M, work units) and geometry.  python3 scripts/plan_stats.py c2 c3 ..."""
import importlib, os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch
import bench
pkg = importlib.import_module("minion-plasmid-consensus_amd")
for cfg in sys.argv[1:]:
    samples, _ = bench.shard_samples(pkg, cfg, 0, 1)
    r = pkg.engine.Runner(samples)
    r.step(0.1, 5.0)
    torch.cuda.synchronize()
    st = [int(x) for x in r.plan.status()]
    print(cfg, "N", sum(len(s["tstart"]) for s in samples), "rows", st[2], "mixed", st[3], "units", st[4], r.plan.info(), flush=True)
