#!/usr/bin/env python3
"""Parse geometry A/B: the parse phase (K_clear + K_parse [+ K_subs]) and the
full step under planner overrides (MPC_PARSE_GEOMETRY="tm,win,nw", read at plan
creation), interleaved in one process, HIP events, medians.  The overrides are
compiled only into the experiment build exp/v/tuning.so (-DMPC_TUNING_OVERRIDES;
build it first with `python3 -c "import _build; _build.build_hip(out='exp/v/tuning.so',
extra=['-DMPC_TUNING_OVERRIDES'])"` from the package directory).
  python3 scripts/geom_ab.py c2:default,2/2048/8,1/1024/8 c3:default,3/2048/8"""
import importlib
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
pkg = importlib.import_module("minion-plasmid-consensus_amd")
eng = pkg.engine
eng.set_library(os.path.join(REPO, "exp", "v", "tuning.so"))
bench = importlib.import_module("bench")


def timed(fn, reps=15):
    st = torch.cuda.current_stream()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record(st)
        fn()
        b.record(st)
    torch.cuda.synchronize()
    return float(np.median([a.elapsed_time(b) for a, b in ev]) * 1e3)


for arg in sys.argv[1:]:
    cfg, geos = arg.split(":")
    samples, _ = bench.shard_samples(pkg, cfg, 0, 1)
    runners = {}
    for g in geos.split(","):
        if g == "default":
            os.environ.pop("MPC_PARSE_GEOMETRY", None)
        else:
            os.environ["MPC_PARSE_GEOMETRY"] = g.replace("/", ",")
        r = eng.Runner(samples)
        r.step(0.1, 5.0)
        r.check()
        runners[g] = r
    os.environ.pop("MPC_PARSE_GEOMETRY", None)
    res = {g: {"parse": [], "step": []} for g in runners}
    for _ in range(3):
        for g, r in runners.items():
            res[g]["parse"].append(timed(lambda: r.plan.phase("parse")))
            res[g]["step"].append(timed(lambda: r.step(0.1, 5.0)))
    for g, r in runners.items():
        r.step(0.1, 5.0)
        r.check()
        i = r.plan.info()
        print(cfg, g, "parse %.1f us" % np.median(res[g]["parse"]), "step %.1f us" % np.median(res[g]["step"]),
              {k: i[k] for k in ("tally_mode", "parse_window", "parse_waves", "parse_workgroups", "parse_lds_bytes")},
              flush=True)
    del runners
    torch.cuda.empty_cache()
