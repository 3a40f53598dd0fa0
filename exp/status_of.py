#!/usr/bin/env python3
"""One step with a variant library, print the status words (experiment counters in words 5-7)."""
import importlib, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
pkg = importlib.import_module("minion-plasmid-consensus_amd")
pkg.engine.set_library(os.path.abspath(sys.argv[1]))
import bench
samples, _ = bench.shard_samples(pkg, os.environ.get("KEXP_CFG", "c2"), 0, 1)
r = pkg.engine.Runner(samples)
r.step(0.1, 5.0)
print("STATUS", [int(x) for x in r.plan.status()], r.plan.info())
