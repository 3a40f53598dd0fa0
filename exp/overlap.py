#!/usr/bin/env python3
"""Batches in flight: K steps of one Runner on one stream vs K steps alternating
over R runners (independent workspaces, same batch data) on R streams, so a
batch's latency-bound post-parse chain can overlap the next batch's parse.
  python3 exp/overlap.py c2 [R ...]     (PARSE_CUS=<n>: parse grid sized for n CUs)"""
import importlib
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

pkg = importlib.import_module("minion-plasmid-consensus_amd")
eng = pkg.engine
if os.environ.get("KEXP_LIB"):
    eng.set_library(os.path.abspath(os.environ["KEXP_LIB"]))  # variant build under test (experiments only)
import bench  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
Rs = [int(x) for x in sys.argv[2:]] or [1, 2, 3]
samples, _ = bench.shard_samples(pkg, cfg, 0, 1)
K = 40
for R in Rs:
    runners = [eng.Runner(samples, parse_cus=int(os.environ.get("PARSE_CUS", "0"))) for _ in range(R)]
    streams = [torch.cuda.Stream() for _ in range(R)]
    for r, s in zip(runners, streams):
        with torch.cuda.stream(s):
            for _ in range(3):
                r.step(0.1, 5.0, s)
    torch.cuda.synchronize()
    best = None
    for _ in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(K):
            i = k % R
            runners[i].step(0.1, 5.0, streams[i])
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / K * 1e6
        best = dt if best is None else min(best, dt)
    for r in runners:
        r.check()
    print(cfg, "batches in flight", R, "us per step %.1f" % best, flush=True)
    del runners
    torch.cuda.empty_cache()
