"""Helpers to read tests/golden/ (fixtures produced by scripts/make_golden.py)."""
import gzip
import json
import os

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

# Documented divergences of the HIP path from the reference (DESIGN.md §6,
# include/mpc.h MPC_DE_UNSUPPORTED): a negative target start whose flank or
# '+' insertion Python's negative index wrap writes into an ODD position (extra
# slots in a reference-base position).  The reference exits 0 (the golden pins
# what it writes; the oracle matches it); the drop-in exits 1 with no outputs.
DIVERGENT = {
    "n_neg_ins": "'+' at a negative coordinate in [-n, 0): slots in wrapped odd position n + i",
    "n_neg_flank": "upstream flank at a negative tstart in [-n, 0): slots in wrapped odd position n + tstart",
    "n_neg_end": "downstream flank of a read ending in [-n, 0): slots appended to a wrapped odd position",
}


def cases():
    return sorted(d for d in os.listdir(GOLDEN) if os.path.isfile(os.path.join(GOLDEN, d, "case.json")))


def read(case, fname):
    p = os.path.join(GOLDEN, case, fname)
    if os.path.exists(p):
        return open(p, "rb").read()
    with gzip.open(p + ".gz", "rb") as f:
        return f.read()


def manifest(case):
    return json.load(open(os.path.join(GOLDEN, case, "case.json")))


def materialize(case, d):
    """Write the case's CLI inputs into directory d; returns (ref, reads, paf) paths."""
    out = []
    for fn in ("ref.fa", "reads.fa", "in.paf"):
        p = os.path.join(d, fn)
        with open(p, "wb") as f:
            f.write(read(case, fn))
        out.append(p)
    return tuple(out)


def runs(case):
    m = manifest(case)
    for k, r in enumerate(m["runs"]):
        exp = {f: read(case, fn) for f, fn in r["files"].items()}
        yield k, r, exp
