#!/usr/bin/env python3
"""Experiments: every variant library gives the first library's calls (a
product build, parity-tested against the oracle), bit for bit, on full-size
configs.  One process, samples generated once per config.
  VCHK_CFGS=c1,c2,c4 python3 scripts/variant_check.py exp/v/head.so exp/v/a.so exp/v/b.so"""
import importlib
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
pkg = importlib.import_module("minion-plasmid-consensus_amd")
eng = pkg.engine
import bench  # noqa: E402

libs = [os.path.abspath(p) for p in sys.argv[1:]]
eng.LIB_PATH = libs[0]
eng.lib()
bad = 0
for cfg in os.environ.get("VCHK_CFGS", "c1,c2,c4").split(","):
    samples, _ = bench.shard_samples(pkg, cfg, 0, 1)
    ref = None
    for p in libs:
        eng._lib = None  # (experiments only) switch the variant
        eng.LIB_PATH = p
        out = []
        for mdf, gtf in ((-1.0, 1.0), (0.1, 5.0)):
            res = eng.pileup(samples, mdf, gtf)
            out.append([{k: np.asarray(v).copy() if not np.isscalar(v) else v for k, v in r.items()} for r in res])
        if ref is None:
            ref = out
            continue
        ok = True
        for a, b in zip(ref, out):
            for ra, rb in zip(a, b):
                for k in ra:
                    if not np.array_equal(np.asarray(ra[k]), np.asarray(rb[k])):
                        ok = False
                        print("  MISMATCH", cfg, os.path.basename(p), k, flush=True)
                        break
        bad += not ok
        print("%s %s %s" % (cfg, os.path.basename(p), "== product" if ok else "DIFFERS"), flush=True)
sys.exit(1 if bad else 0)
