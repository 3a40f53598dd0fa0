#!/usr/bin/env python3
"""Batches in flight with the parse and the post-parse chain on CU-masked
streams (hipExtStreamCreateWithCUMask): K_parse holds every VGPR of a CU, so a
chain block resident on a CU keeps the next parse workgroup off it; masking
gives each its own CUs.  Per pipeline: a parse stream and a chain stream
ordered by events.  Modes:
  run      one stream per pipeline, mpc_run (bench.py's loop)
  split    parse / chain on two plain streams per pipeline
  mask:K   parse on the CUs with (cu >> 3) % K != K - 1, chain on the rest
Every pipeline's calls are compared with pipeline 0's after the timed steps.

  python3 exp/cusplit.py c2 3 run split mask:4 mask:8
"""
import ctypes
import importlib
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
pkg = importlib.import_module("minion-plasmid-consensus_amd")
eng = pkg.engine
bench = importlib.import_module("bench")
hip = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
CHAIN = ("index", "runs", "tally", "layout", "rows")


def cu_stream(pred, ncu):
    words = [0] * ((ncu + 31) // 32)
    for i in range(ncu):
        if pred(i):
            words[i // 32] |= 1 << (i % 32)
    s = ctypes.c_void_p()
    arr = (ctypes.c_uint32 * len(words))(*words)
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), ctypes.c_uint32(len(words)), arr)
    if rc != 0:
        raise RuntimeError("hipExtStreamCreateWithCUMask: %d" % rc)
    return torch.cuda.ExternalStream(s.value)


def main():
    cfg, R, modes = sys.argv[1], int(sys.argv[2]), sys.argv[3:]
    steps, warm = int(os.environ.get("CUS_STEPS", "200")), int(os.environ.get("CUS_WARMUP", "20"))
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    samples, _ = bench.shard_samples(pkg, cfg, 0, 1)
    mdf, gtf = 0.1, 5.0
    for mode in modes:
        if mode.startswith("mask:"):
            k = int(mode.split(":")[1])
            par = lambda i, k=k: (i >> 3) % k != k - 1
            pcus = sum(1 for i in range(ncu) if par(i))
        else:
            pcus = bench.PARSE_CUS_INFLIGHT[cfg]
        runners = [eng.Runner(samples, parse_cus=pcus) for _ in range(R)]
        for r in runners:
            r.step(mdf, gtf)
        torch.cuda.synchronize()
        if mode == "run":
            st = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(R - 1)]

            def step(k):
                runners[k % R].plan.run(mdf, gtf, st[k % R])
        else:
            if mode == "split":
                ps = [torch.cuda.Stream() for _ in range(R)]
                cs = [torch.cuda.Stream() for _ in range(R)]
            else:
                ps = [cu_stream(par, ncu) for _ in range(R)]
                cs = [cu_stream(lambda i, par=par: not par(i), ncu) for _ in range(R)]
            parsed = [torch.cuda.Event() for _ in range(R)]
            done = [torch.cuda.Event() for _ in range(R)]
            for e, s in zip(done, cs):
                e.record(s)

            def step(k):
                p = k % R
                plan = runners[p].plan
                ps[p].wait_event(done[p])
                plan.phase("parse", ps[p])
                parsed[p].record(ps[p])
                cs[p].wait_event(parsed[p])
                for ph in CHAIN:
                    plan.phase(ph, cs[p])
                plan.phase("consensus", cs[p], mdf, gtf)
                done[p].record(cs[p])
        for k in range(warm):
            step(k)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(steps):
            step(k)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        ref = runners[0].plan.fetch()
        same = all(_same(r.plan.fetch(), ref) for r in runners[1:])
        for r in runners:
            r.check()
        print("%s R=%d %-8s parse_cus %3d: %.1f us per step, calls identical across pipelines: %s"
              % (cfg, R, mode, pcus, dt * 1e6 / steps, same), flush=True)
        del runners
        torch.cuda.synchronize()


def _same(a, b):
    for x, y in zip(a, b):
        for key in x:
            if isinstance(x[key], np.ndarray):
                if not np.array_equal(x[key], y[key]):
                    return False
            elif x[key] != y[key]:
                return False
    return True


if __name__ == "__main__":
    main()
