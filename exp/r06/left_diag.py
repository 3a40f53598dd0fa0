#!/usr/bin/env python3
"""K_left event paths of one single-batch step (diagnostic build exp/v/leftdiag.so):
   KEXP_CFG=c3 python3 exp/r06/left_diag.py exp/v/leftdiag.so"""
import ctypes
import importlib
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
pkg = importlib.import_module("minion-plasmid-consensus_amd")
eng = pkg.engine
import bench  # noqa: E402

cfg = os.environ.get("KEXP_CFG", "c3")
eng.LIB_PATH = os.path.abspath(sys.argv[1])
L = eng.lib()
samples, _ = bench.shard_samples(pkg, cfg, 0, 1)
plan = eng.Plan(eng.Batch(samples))
plan.run(0.1, 5.0)
torch.cuda.synchronize()
out = (ctypes.c_ulonglong * 8)()
L.mpc_diag_left(out, 1)
plan.run(0.1, 5.0)
torch.cuda.synchronize()
L.mpc_diag_left(out, 0)
ev, srch, k8, rng, k16, k32 = out[0], out[1], out[2], out[3], out[4], out[5]
print("%s events %d  mixed-gap (searched) %.1f %%  mean range %.1f  k>=8 %.1f %%  k>=16 %.1f %%  k>=32 %.1f %%" % (
    cfg, ev, 100.0 * srch / max(ev, 1), rng / max(srch, 1), 100.0 * k8 / max(ev, 1), 100.0 * k16 / max(ev, 1),
    100.0 * k32 / max(ev, 1)))
