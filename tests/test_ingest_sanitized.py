"""ASan + UBSan build of the native host I/O (csrc/ingest.cpp, writers.cpp,
pseudopair.cpp):
a driver executable (tests/native/ingest_driver.cpp) built with
-fsanitize=address,undefined and no recovery runs over every golden input, the
edge / error / declined cases of test_ingest_native.py and synthetic files
with 1 and 8 threads.  Any sanitizer report fails the run (non-zero exit); the
digests of its outputs must equal those of the production library (CPU only)."""
import importlib
import os
import shutil
import subprocess

import numpy as np
import pytest

import golden_util as gu
import test_ingest_native as tin

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(REPO, "build", "ingest_asan")


def _fnv(a):
    b = np.ascontiguousarray(a).view(np.uint8)
    h = 1469598103934665603
    # vectorless FNV-1a on small arrays; large ones are hashed in chunks of the same function
    for x in b.tobytes():
        h ^= x
        h = (h * 1099511628211) & 0xFFFFFFFFFFFFFFFF
    return "%016x" % h


@pytest.fixture(scope="module")
def asan_bin():
    if shutil.which("g++") is None:
        pytest.skip("no g++")
    os.makedirs(os.path.dirname(BIN), exist_ok=True)
    src = [os.path.join(REPO, "minion-plasmid-consensus_amd", "csrc", f) for f in
           ("ingest.cpp", "writers.cpp", "pseudopair.cpp")] + [os.path.join(REPO, "tests", "native", "ingest_driver.cpp")]
    # build under a per-process name, then rename: pytest-xdist workers each
    # build it, and one must never exec a file another is still writing
    tmp = "%s.%d" % (BIN, os.getpid())
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
                    "-fno-sanitize-recover=all", "-pthread", "-I", os.path.join(REPO, "include"), "-o", tmp] + src,
                   check=True)
    os.replace(tmp, BIN)
    return BIN


def _expect(ing, ref, paf, reads):
    try:
        r = ing.pack_sample_native(ref, paf, reads)
    except ing.IngestError:
        return "1"
    if r is None:
        return "2"
    n = len(r["tstart"])
    parts = ["0", str(n), str(r["n_alignments"])]
    for k in ("ref", "cs", "cs_off", "tstart", "up", "up_off", "down", "down_off", "aligned"):
        parts.append(f"{k}={_fnv(r[k])}")
    return " ".join(parts)


def _run(asan_bin, ing, ref, paf, reads, threads=(1, 8)):
    exp = _expect(ing, ref, paf, reads)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:exitcode=86",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1:exitcode=87")
    for t in threads:
        p = subprocess.run([asan_bin, ref, paf, reads, str(t)], capture_output=True, text=True, env=env, timeout=120)
        assert p.returncode == 0, (ref, t, p.returncode, p.stderr[-2000:])
        got = p.stdout.strip()
        if exp in ("1", "2"):
            assert got.split()[0] == exp, (ref, got)
        else:
            assert got == exp, (ref, t)


@pytest.fixture(scope="module")
def ing():
    return importlib.import_module("minion-plasmid-consensus_amd.ingest")


def test_golden_inputs_sanitized(asan_bin, ing, tmp_path):
    for case in gu.cases():
        d = tmp_path / case
        d.mkdir()
        ref, reads, paf = gu.materialize(case, str(d))
        _run(asan_bin, ing, ref, paf, reads)


def test_edge_error_declined_sanitized(asan_bin, ing, tmp_path):
    for table in (tin.EDGE, tin.ERRORS, tin.DECLINED):
        for name, files in table.items():
            d = tmp_path / name
            d.mkdir()
            _run(asan_bin, ing, *tin._files(d, *files))


def test_synthetic_sanitized(asan_bin, ing, tmp_path):
    syn = importlib.import_module("minion-plasmid-consensus_amd.synth").Synth(
        n=800, n_reads=600, profile="indel", seed=19, frac_partial=0.4, flank=(0, 120))
    p = {k: str(tmp_path / k) for k in ("ref.fa", "reads.fa", "s.paf", "ras.fa", "as.paf")}
    syn.write_files(p["ref.fa"], p["reads.fa"], p["s.paf"], p["ras.fa"], p["as.paf"])
    _run(asan_bin, ing, p["ref.fa"], p["s.paf"], p["reads.fa"], threads=(1, 3, 8))
    _run(asan_bin, ing, p["ras.fa"], p["as.paf"], p["reads.fa"])


def _san_env():
    return dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:exitcode=86",
                UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1:exitcode=87")


def test_writers_sanitized(asan_bin, tmp_path):
    w = importlib.import_module("minion-plasmid-consensus_amd.writers")
    for n in (0, 1, 5000, 40000):
        outs = [str(tmp_path / ("%s%d" % (x, n))) for x in ("c", "ch", "acc")]
        p = subprocess.run([asan_bin, "writecalls", str(n), "7", *outs], capture_output=True, text=True,
                           env=_san_env(), timeout=120)
        assert p.returncode == 0 and p.stdout.strip() == "0", (n, p.stderr[-2000:])
        assert open(outs[0]).read().startswith(">consensus\n")
        assert open(outs[1]).read().count("\n") == 1 + 2 * n
    assert w is not None


def test_pseudopair_sanitized(asan_bin, tmp_path):
    import test_pseudopair as tp
    pp = importlib.import_module("minion-plasmid-consensus_amd.pseudopair_reads")
    for case in tp.cases():
        paf = tmp_path / (case + ".paf")
        paf.write_bytes(tp.read(case, "in.paf"))
        out = tmp_path / (case + ".out")
        p = subprocess.run([asan_bin, "pseudopair", str(paf), "0", str(out)], capture_output=True, text=True,
                           env=_san_env(), timeout=120)
        assert p.returncode == 0, (case, p.stderr[-2000:])
        status = int(p.stdout.split()[0])
        try:
            st = pp.pseudopair_native(str(paf), 0, str(tmp_path / "ref.out"))
            exp = 2 if st is None else 0
        except pp.PairError:
            exp = 1
        assert status == exp, case
