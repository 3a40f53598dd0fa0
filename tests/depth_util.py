"""Helpers for the depth-scale parity tests (test infrastructure).

``oracle_many`` runs the C oracle (oracle/mpc_oracle.c) on several samples at
once: ctypes releases the GIL during the foreign call, so samples run on
separate host threads (the oracle itself is the single-threaded restatement).

``derive`` turns one FULL-pileup oracle result (min_depth_factor = -1,
global_threshold_factor = 1: every slot is emitted and the called base equals
the pre-GTF chromatogram base) into the result for any (mdf, gtf), by the two
tests of the reference's Step 6 (mapped_paf_read_parser.py:421 and :428) in
float64 -- so one oracle pass checks every threshold pair.
tests/test_depth_cpu.py checks ``derive`` against direct oracle runs.
"""
import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np

import oracle

KEYS = ("base", "chrom1", "chrom2", "count", "count2", "total")


def oracle_one(s, mdf, gtf):
    return oracle.run_packed(s["ref"], s["cs"], s["cs_off"], s["tstart"], s["up"], s["up_off"], s["down"],
                             s["down_off"], mdf, gtf)


def oracle_many(samples, mdf, gtf, threads=None):
    threads = threads or min(len(samples), 16, os.cpu_count() or 1)
    with ThreadPoolExecutor(max_workers=max(1, threads)) as ex:
        return list(ex.map(lambda s: oracle_one(s, mdf, gtf), samples))


def derive(full, mdf, gtf):
    """The (mdf, gtf) result from a full-pileup (mdf=-1, gtf=1) result."""
    cnt = np.asarray(full["count"], dtype=np.int64)
    cnt2 = np.asarray(full["count2"], dtype=np.int64)
    thr = float(full["max_depth"]) * float(mdf)                      # :338 DEPTH_THRESHOLD
    with np.errstate(invalid="ignore"):  # inf * 0 = nan compares False, as in Python
        keep = cnt.astype(np.float64) > thr                          # :428 count > DEPTH_THRESHOLD
        weak = cnt.astype(np.float64) < float(gtf) * cnt2.astype(np.float64)  # :421 count < GTF * count2
    base = np.where(weak, np.uint8(ord("N")), np.asarray(full["chrom1"], dtype=np.uint8))
    out = {"base": base[keep], "max_depth": int(full["max_depth"])}
    for k in ("chrom1", "chrom2", "count", "count2", "total"):
        out[k] = np.asarray(full[k])[keep]
    return out


def compare(got, exp, tag):
    assert got["max_depth"] == exp["max_depth"], (tag, got["max_depth"], exp["max_depth"])
    for k in KEYS:
        a = np.asarray(got[k], dtype=np.int64)
        b = np.asarray(exp[k], dtype=np.int64)
        assert a.shape == b.shape, (tag, k, a.shape, b.shape)
        if not np.array_equal(a, b):
            bad = np.nonzero(a != b)[0][:5]
            raise AssertionError(f"{tag} {k} differs at {bad.tolist()}: {a[bad].tolist()} vs {b[bad].tolist()}")
