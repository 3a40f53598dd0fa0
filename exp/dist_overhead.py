#!/usr/bin/env python3
"""Cost of the distributed step path at WORLD_SIZE=1 on one GPU (RCCL):
device time per step and host enqueue time per step, for the plain Runner,
ShardedPileup + DistExchange on one communicator, and one communicator per
pipeline (dist.new_group), with 1 and 2 pipelines in flight.
  torchrun --nproc-per-node 1 exp/dist_overhead.py [cfg]"""
import importlib
import os
import sys
import time

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
K = 40


def run(name, runners):
    R = len(runners)
    streams = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(R - 1)]
    for k in range(3 * R):
        with torch.cuda.stream(streams[k % R]):
            runners[k % R].step(0.1, 5.0)
    torch.cuda.synchronize()
    host = 0.0
    t0 = time.perf_counter()
    for k in range(K):
        h0 = time.perf_counter()
        with torch.cuda.stream(streams[k % R]):
            runners[k % R].step(0.1, 5.0)
        host += time.perf_counter() - h0
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    for r in runners:
        r.check()
    print("%-34s R=%d  %.1f us/step   host enqueue %.1f us/step" % (name, R, dt / K * 1e6, host / K * 1e6), flush=True)


cus = bench.PARSE_CUS_INFLIGHT[cfg]
run("Runner", [pkg.engine.Runner(samples)])
run("Runner", [pkg.engine.Runner(samples, parse_cus=cus) for _ in range(2)])
ex = dmod.DistExchange()
run("Sharded, one communicator", [dmod.ShardedPileup([samples], [0], ex=ex)])
run("Sharded, one communicator", [dmod.ShardedPileup([samples], [0], ex=ex, parse_cus=cus) for _ in range(2)])
groups = [dist.new_group(list(range(dist.get_world_size()))) for _ in range(2)]
run("Sharded, communicator per pipeline",
    [dmod.ShardedPileup([samples], [0], ex=dmod.DistExchange(g), parse_cus=cus) for g in groups])
dist.destroy_process_group()
