#!/usr/bin/env python3
"""The distributed step captured in a HIP graph (torch.cuda.graph) at
WORLD_SIZE=1 over RCCL: every phase launch, torch glue op and collective of
ShardedPileup.step replayed without host dispatch.  Eager vs graph: device
time per step, host time per step, identical calls.
  torchrun --nproc-per-node 1 exp/dist_graph.py [cfg]"""
import importlib
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
pkg = importlib.import_module("minion-plasmid-consensus_amd")
dmod = importlib.import_module("minion-plasmid-consensus_amd.dist")
bench = importlib.import_module("bench")
samples, _ = bench.shard_samples(pkg, cfg, 0, 1)
cus = bench.PARSE_CUS_INFLIGHT[cfg]
K = 40
groups = [dist.new_group(list(range(dist.get_world_size()))) for _ in range(2)]
pipes = [dmod.ShardedPileup([samples], [0], ex=dmod.DistExchange(g), parse_cus=cus) for g in groups]
streams = [torch.cuda.Stream() for _ in pipes]
for k in range(6):
    with torch.cuda.stream(streams[k % 2]):
        pipes[k % 2].step(0.1, 5.0)
torch.cuda.synchronize()
ref = [p.fetch() for p in pipes]


def timed(label, fn):
    torch.cuda.synchronize()
    host = 0.0
    t0 = time.perf_counter()
    for k in range(K):
        h0 = time.perf_counter()
        fn(k)
        host += time.perf_counter() - h0
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print("%-28s %.1f us/step   host %.1f us/step" % (label, dt / K * 1e6, host / K * 1e6), flush=True)


def eager(k):
    with torch.cuda.stream(streams[k % 2]):
        pipes[k % 2].step(0.1, 5.0)


timed("eager, 2 pipelines", eager)
graphs = []
for p, s in zip(pipes, streams):
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        p.step(0.1, 5.0)  # (warm: allocations of the glue ops)
        torch.cuda.current_stream().synchronize()
        with torch.cuda.graph(g, stream=s):
            p.step(0.1, 5.0)
    graphs.append(g)
torch.cuda.synchronize()
print("captured", flush=True)


def replay(k):
    with torch.cuda.stream(streams[k % 2]):
        graphs[k % 2].replay()


timed("graph, 2 pipelines", replay)
for p, r in zip(pipes, ref):
    p.check()
    got = p.fetch()
    for a, b in zip(got, r):
        assert all(np.array_equal(a[key], b[key]) for key in ("base", "count", "count2", "total")), "graph replay differs"
print("graph replay equals eager", flush=True)
dist.destroy_process_group()
