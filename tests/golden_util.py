"""Helpers to read tests/golden/ (fixtures produced by scripts/make_golden.py)."""
import gzip
import json
import os

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

# Documented divergences of the HIP path from the reference.
# Since round 6 the three negative-target-start cases whose strings Python's
# negative index wrap writes into an ODD position (n_neg_ins, n_neg_flank,
# n_neg_end) are replayed on the device (K_woprep .. K_worows) and match.
# What remains: references past the engine's coordinate scheme (include/mpc.h,
# n <= 2^22 - 2).  The reference exits 0 (the golden pins what it writes; the
# oracle matches it); the drop-in exits 1 with no outputs.
DIVERGENT = {
    "l_ref_past_limit": "reference of 2^22 - 1 bases: past the 32-bit coordinate scheme (mpc_plan_create MPC_E_ARG)",
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
