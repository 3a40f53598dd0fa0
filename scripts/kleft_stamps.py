#!/usr/bin/env python3
"""Where K_left's waves spend their cycles: the -DMPC_STAMPS_LEFT diagnostic
build (s_memtime stamps around K_left's per-unit segments, summed per wave) on
one bench.py workload.  Read the SHARES, not the totals: the stamps' own
lgkmcnt(0) waits forbid overlaps the product kernel has.

  hipcc ... -DMPC_STAMPS_LEFT -o exp/v/lstamps.so
  python3 scripts/kleft_stamps.py exp/v/lstamps.so c3 [c2 ...]
"""
import ctypes
import importlib
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

SEGS = ["unit: LDS clear", "unit: record + tables (2 round trips, scan)", "unit: event loads + RIGHT-read stage issued",
        "unit: barrier (loads land)", "unit: tally (LDS atomics)", "unit: barrier after tally",
        "unit: flush (global atomics) + barrier", "per-read pass (long insertions, upstream flanks)"]


def main():
    lib, cfgs = sys.argv[1], sys.argv[2:] or ["c3"]
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
        r = eng.Runner(samples)
        for _ in range(3):
            r.step(0.1, 5.0)
        torch.cuda.synchronize()
        assert L.mpc_debug_stamps_clear() == 0
        r.step(0.1, 5.0)
        torch.cuda.synchronize()
        st = [int(x) for x in r.plan.status()]
        buf = np.zeros((1 << 16) * 8, dtype=np.uint64)
        assert L.mpc_debug_stamps(buf.ctypes.data, buf.size) == 0
        per = buf.reshape(-1, 8).astype(np.float64)
        per = per[per.sum(axis=1) > 0]
        tot = per.sum(axis=0)
        rec = {"config": cfg, "waves": int(len(per)), "units": st[4],
               "mean_cycles_per_wave": float(per.sum(axis=1).mean()),
               "max_cycles_per_wave": float(per.sum(axis=1).max()),
               "segments": {n: {"share": float(t / tot.sum()), "mean_cycles_per_wave": float(t / len(per))}
                            for n, t in zip(SEGS, tot)}}
        out[cfg] = rec
        print(cfg, "units", st[4], "waves", len(per), "mean cycles/wave %.0f max %.0f"
              % (rec["mean_cycles_per_wave"], rec["max_cycles_per_wave"]))
        for n, t in zip(SEGS, tot):
            print("   %-52s %6.1f %%  %10.0f cyc/wave" % (n, 100 * t / tot.sum(), t / len(per)))
        del r
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    with open(os.path.join(REPO, "gpurun_out", "kleft_stamps.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
