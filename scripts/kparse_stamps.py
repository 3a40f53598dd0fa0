#!/usr/bin/env python3
"""Where K_parse's waves spend their cycles: the -DMPC_STAMPS diagnostic build
(s_memtime stamps around the kernel's segments, summed per wave) on one
bench.py workload.  Read the SHARES, not the totals: the stamps' own
lgkmcnt(0) waits forbid overlaps the product kernel has.

  hipcc ... -DMPC_STAMPS -o build/variants/stamps.so   (scripts/build_variants.sh stamps=-DMPC_STAMPS)
  python3 scripts/kparse_stamps.py build/variants/stamps.so c2 [c3 ...]
"""
import ctypes
import importlib
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

SEGS = ["window: fetch wait", "window: classes + cut + unit list", "round: decode", "round: scan + base",
        "round: effects", "window tail + reads ending", "pre-epilogue barrier wait", "epilogue"]


def main():
    lib, cfgs = sys.argv[1], sys.argv[2:] or ["c2"]
    import torch
    pkg = importlib.import_module("minion-plasmid-consensus_amd")
    eng = pkg.engine
    eng.set_library(os.path.abspath(lib))
    L = eng.lib()
    L.mpc_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    L.mpc_debug_stamps.restype = ctypes.c_int
    L.mpc_debug_stamps_clear.restype = ctypes.c_int
    bench = importlib.import_module("bench")
    out = {}
    for cfg in cfgs:
        samples, _ = bench.shard_samples(pkg, cfg, 0, 1)
        plan = eng.Plan(eng.Batch(samples))
        for _ in range(3):
            plan.phase("parse")
        torch.cuda.synchronize()
        assert L.mpc_debug_stamps_clear() == 0
        plan.phase("parse")
        torch.cuda.synchronize()
        info = plan.info()
        nw = info["parse_workgroups"] * 16
        buf = np.zeros(nw * 8, dtype=np.uint64)
        assert L.mpc_debug_stamps(buf.ctypes.data, buf.size) == 0
        per = buf.reshape(-1, 8)[: info["parse_workgroups"] * 16].astype(np.float64)
        per = per[per.sum(axis=1) > 0]
        tot = per.sum(axis=0)
        rec = {"config": cfg, "waves": int(len(per)), "geometry": info,
               "mean_cycles_per_wave": float(per.sum(axis=1).mean()),
               "segments": {n: {"share": float(t / tot.sum()), "mean_cycles_per_wave": float(t / len(per))}
                            for n, t in zip(SEGS, tot)}}
        out[cfg] = rec
        print(cfg, "waves", len(per), "mean cycles/wave %.0f" % rec["mean_cycles_per_wave"])
        for n, t in zip(SEGS, tot):
            print("   %-36s %6.1f %%  %10.0f cyc/wave" % (n, 100 * t / tot.sum(), t / len(per)))
        del plan
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    with open(os.path.join(REPO, "gpurun_out", "kparse_stamps.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
