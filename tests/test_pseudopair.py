"""Drop-in pseudopair_reads (rule pseudopair_reads, Snakefile:211-228) against the
reference script's own outputs (tests/golden_pseudopair, scripts/make_golden_pseudopair.py),
through the CLI, with the native parser (csrc/pseudopair.cpp) and with the Python
restatement; plus randomized duplicate-heavy PAFs, native vs Python.  CPU only."""
import gzip
import importlib
import json
import os
import random

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.join(HERE, "golden_pseudopair")


def cases():
    return sorted(d for d in os.listdir(ROOT) if os.path.exists(os.path.join(ROOT, d, "case.json")))


def read(case, fn):
    p = os.path.join(ROOT, case, fn)
    if os.path.exists(p):
        return open(p, "rb").read()
    return gzip.open(p + ".gz", "rb").read()


@pytest.fixture(scope="module")
def pp():
    return importlib.import_module("minion-plasmid-consensus_amd.pseudopair_reads")


NATIVE_DECLINES = {"py_int_forms", "crlf", "bad_int"}  # Python int() forms / universal newlines: Python decides


@pytest.mark.parametrize("case", cases())
@pytest.mark.parametrize("path", ["native", "python"])
def test_matches_reference(pp, case, path, tmp_path, monkeypatch):
    paf = tmp_path / "in.paf"
    paf.write_bytes(read(case, "in.paf"))
    if path == "python":
        monkeypatch.setattr(pp, "pseudopair_native", lambda *a, **k: None)
    elif case not in NATIVE_DECLINES:
        # the native parser decides this input itself (no fallback)
        try:
            st = pp.pseudopair_native(str(paf), 0, str(tmp_path / "probe.txt"))
            assert st is not None, case
        except pp.PairError:
            pass
    runs = json.load(open(os.path.join(ROOT, case, "case.json")))["runs"]
    for k, run in enumerate(runs):
        out = tmp_path / f"o{k}.txt"
        argv = ["--paf", str(paf), "--pseudopairs", str(out)]
        if run["min_align_length"] is not None:
            argv += ["--min_align_length", str(run["min_align_length"])]
        rc = pp.main(argv)
        assert rc == run["exit"], (case, k)
        if run["file"] is None:
            assert not out.exists(), (case, k)
        else:
            assert out.read_bytes() == read(case, run["file"]), (case, k)


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_random_native_vs_python(pp, seed, tmp_path):
    rng = random.Random(seed)
    lines = []
    names = ["r%d" % rng.randint(0, 400) for _ in range(3000)]  # heavy repetition: delete / re-add chains
    for nm in names:
        qlen = rng.randint(1, 5000)
        qs, qe = rng.randint(0, qlen), rng.randint(0, qlen)
        nf = rng.choice([5, 6, 13])
        f = [nm, str(qlen), str(qs), str(qe), rng.choice(["+", "-", "+"])] + ["x"] * (nf - 5)
        lines.append("\t".join(f) + "\n")
    text = "".join(lines)
    if seed == 2:
        text = text.rstrip("\n")  # last line without a newline
    paf = tmp_path / "in.paf"
    paf.write_text(text)
    for m in (0, 1500, 4000):
        st = pp.pseudopair_native(str(paf), m, str(tmp_path / "n.txt"))
        assert st is not None
        pairs, nf, nr, nfk, nrk = pp.pseudopair_python(str(paf), m)
        assert (st.n_fwd, st.n_rev, st.n_fwd_kept, st.n_rev_kept) == (nf, nr, nfk, nrk)
        assert (tmp_path / "n.txt").read_text() == "".join("%s %s\n" % x for x in pairs)
