"""The C-ABI library loads and exports every function declared in include/mpc.h
(no compute calls: runs without a GPU)."""
import ctypes
import os
import re
import subprocess
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared(header="mpc.h"):
    txt = open(os.path.join(REPO, "include", header)).read()
    return sorted(set(re.findall(r"^(?:int|void|size_t|const char\*)\s+(mpc_\w+)\(", txt, re.M)))


def test_header_declares_entry_points():
    names = declared()
    for f in ("mpc_version", "mpc_plan_create", "mpc_plan_bind", "mpc_parse", "mpc_index", "mpc_runs", "mpc_tally",
              "mpc_layout", "mpc_rows", "mpc_consensus", "mpc_run", "mpc_profile_kernel"):
        assert f in names


def test_library_exports_all(pkg):
    pkg._build.build_hip()
    lib = pkg.engine.lib()  # (a bare CDLL would map the system HIP runtime beside PyTorch's)
    for name in declared():
        assert hasattr(lib, name), name
    lib.mpc_version.restype = ctypes.c_int
    assert lib.mpc_version() == pkg.engine.ABI_VERSION == 9


def test_no_oracle_in_product():
    """The product package never imports the CPU oracle."""
    pkgdir = os.path.join(REPO, "minion-plasmid-consensus_amd")
    for root, _, files in os.walk(pkgdir):
        for f in files:
            if f.endswith((".py", ".hip", ".cpp", ".h")):
                src = open(os.path.join(root, f), errors="replace").read()
                assert "import oracle" not in src and "mpc_oracle" not in src, f


def test_ingest_library_exports_all(pkg):
    path = pkg._build.build_ingest()
    lib = ctypes.CDLL(path)
    names = declared("mpc_ingest.h")
    assert "mpc_ingest" in names and "mpc_ingest_free" in names
    for name in names:
        assert hasattr(lib, name), name


def test_planner_geometry(pkg):
    """Host-only planning (no device work): every BASELINE config runs K_parse
    with its per-position state in LDS (tally modes 1-3), within the LDS and
    wave budgets, and the reads-per-workgroup cap that keeps the 16-bit LDS
    tallies exact (mpc_kernels.hip wg_reads_cap) holds."""
    g = pkg.engine.geometry
    c2 = g([2686, 2686], [100_000, 100_000], 63 << 20)
    assert c2["tally_mode"] == 1 and c2["max_reads_per_workgroup"] <= c2["reads_per_workgroup_cap"] == 32767
    c3 = g([10_000], [1_000_000], 1200 << 20)
    c4 = g([10_000] * 2, [100_000] * 2, 1070 << 20)
    c5 = g([30_000] * 24, [10_000] * 24, 24 * 3600 * 10_000 // 100)
    assert c5["tally_mode"] == 3  # 30 kb: only the 2-byte depth tallies fit beside the waves
    # the cap binds: 4.9 M tiny reads beside one 10 kb sample fill workgroups to the cap
    st = g([10_000, 30], [100, 16383 * 300], 16383 * 300 * 12)
    assert st["max_reads_per_workgroup"] == st["reads_per_workgroup_cap"]
    for info in (c2, c3, c4, c5, st):
        assert info["tally_mode"] in (1, 2, 3)
        assert info["max_reads_per_workgroup"] <= info["reads_per_workgroup_cap"]
        assert info["reads_per_workgroup_cap"] == (32767 if info["tally_mode"] == 1 else 16383)
        assert info["parse_lds_bytes"] <= 160 * 1024 and info["parse_waves"] in (8, 10, 12, 16)


def test_planner_deferred_placement(pkg):
    """K_parse queues insertion events per wave in LDS (mpc_kernels.hip
    MPC_DEFER_PLACE) only with 2 KiB windows in tally mode 1 or 3 with one
    substitution window, and only when the queues fit the LDS budget without
    changing the geometry: C2-C4 take it, C1 and C5 (LDS full) do not; reads
    with negative starts keep inline placement (the plan binds that K_parse)."""
    g = pkg.engine.geometry
    on = [g([2686, 2686], [100_000, 100_000], 63 << 20), g([10_000], [1_000_000], 1200 << 20),
          g([10_000] * 2, [100_000] * 2, 1070 << 20)]
    off = [g([5000], [20_000], 20_000 * 600), g([30_000] * 24, [10_000] * 24, 24 * 3600 * 10_000 // 100)]
    for info in on:
        assert info["deferred_placement"] == 1 and info["parse_window"] == 2048
        assert info["tally_mode"] in (1, 3) and info["parse_lds_bytes"] <= 160 * 1024
    for info in off:
        assert info["deferred_placement"] == 0
    neg = g([2686, 2686], [100_000, 100_000], 63 << 20, neg_reads=1)
    assert neg["deferred_placement"] == 0
    assert 0 <= on[0]["parse_lds_bytes"] - 16 * 128 * 8 - neg["parse_lds_bytes"] < 16  # (16-byte aligned queues)


def test_planner_parse_cus(pkg):
    """mpc_input.parse_cus (bench.py with batches in flight): the parse grid is
    one balanced wave of resident workgroups on that many CUs -- fewer
    workgroups than the all-CU plan, same geometry otherwise, caps still held;
    0 and out-of-range values mean all 256 CUs."""
    g = pkg.engine.geometry
    shapes = [([2686, 2686], [100_000, 100_000], 63 << 20), ([10_000], [1_000_000], 1200 << 20),
              ([30_000] * 24, [10_000] * 24, 24 * 3600 * 10_000 // 100)]
    for args in shapes:
        full = g(*args)
        assert g(*args, parse_cus=256) == full and g(*args, parse_cus=-3) == full
        prev = full["parse_workgroups"]
        for cus in (224, 160, 128):
            info = g(*args, parse_cus=cus)
            for k in ("tally_mode", "parse_window", "parse_waves", "reads_per_workgroup_cap"):
                assert info[k] == full[k], (args, cus, k)
            assert info["parse_workgroups"] <= min(prev, cus)  # one 16-wave workgroup per CU
            assert info["max_reads_per_workgroup"] <= info["reads_per_workgroup_cap"]
            prev = info["parse_workgroups"]
        assert prev < full["parse_workgroups"]


def test_planner_reference_limit(pkg):
    """The longest reference whose parse state fits LDS (tally mode 0 with the
    fewest waves; ~314 kb); one base beyond it the parse keeps that state in HBM
    (tally mode 4), up to 2^22 - 2 (mpc.h: 32-bit coordinates, 22-bit event
    gaps); past that mpc_plan_create fails (host-only)."""
    g = pkg.engine.geometry
    lo, hi = 100_000, 1_000_000  # bisect the last LDS-state length
    while hi - lo > 1:
        mid = (lo + hi) // 2
        if g([mid], [12], mid * 3)["tally_mode"] == 4:
            hi = mid
        else:
            lo = mid
    assert 250_000 < lo < 400_000, lo
    info = g([lo], [12], lo * 3)
    assert info["tally_mode"] == 0 and info["parse_lds_bytes"] <= 160 * 1024
    big = g([lo + 1], [12], (lo + 1) * 3)
    assert big["tally_mode"] == 4 and big["parse_lds_bytes"] <= 160 * 1024
    top = g([(1 << 22) - 2], [12], (1 << 22) * 3)
    assert top["tally_mode"] == 4
    with pytest.raises(pkg.engine.MpcError):
        g([(1 << 22) - 1], [12], (1 << 22) * 3)


@pytest.mark.parametrize("shape", [
    ([2686, 2686], [100_000, 100_000]),  # C2
    ([10_000], [200_000]),               # C3 shape, fewer reads
    ([30_000] * 6, [10_000] * 6),        # C5 shape, fewer runs
    ([500, 40_000], [37, 3]),            # ragged: fewer reads than waves
])
def test_parse_split(pkg, shape):
    """Host-only: the parse work split (mpc_plan_parse_tables).  Workgroups
    cover every sample's reads once, in order; each workgroup's chunks are a
    contiguous, ordered cut of its reads (at most 3 per wave, include/mpc.h
    MPC_PARSE_CHUNKS bound); the first group of chunks carries about 5/8 of
    the workgroup's cs bytes and the last ones the smallest share."""
    e = pkg.engine
    ref_lens, counts = shape
    rng = np.random.default_rng(7)
    lens = rng.integers(20, 4000, size=sum(counts)) * rng.choice([1, 1, 1, 9], size=sum(counts))
    off = np.concatenate([[0], np.cumsum(lens)])
    work, ch = e.parse_split(ref_lens, counts, off)
    info = e.geometry(ref_lens, counts, int(off[-1]))
    nw = info["parse_waves"]
    rb = np.concatenate([[0], np.cumsum(counts)])
    for s in range(len(counts)):
        w = work[work[:, 0] == s]
        assert w[0, 1] == rb[s] and w[-1, 2] == rb[s + 1]
        assert (w[1:, 1] == w[:-1, 2]).all() and (w[:, 2] > w[:, 1]).all()
    for (s, a, b, nch), c in zip(work, ch):
        assert 1 <= nch <= min(3 * nw, e.PARSE_CHUNKS)
        cb = c[: nch + 1]
        assert cb[0] == a and cb[-1] == b and (np.diff(cb) >= 0).all()
        assert (c[nch:] == b).all()  # padding repeats the end
        if b - a >= 8 * nw and nch == 3 * nw:
            tot = off[b] - off[a]
            first = off[cb[nw]] - off[a]
            assert 0.45 * tot <= first <= 0.8 * tot, (first, tot)


def _integration_fields():
    """Field names of the mpc_input ctypes class in INTEGRATION.md's binding."""
    txt = open(os.path.join(REPO, "INTEGRATION.md")).read()
    m = re.search(r"class mpc_input\(ctypes\.Structure\):.*?_fields_ = \[(.*?)\n\n", txt, re.S)
    assert m, "INTEGRATION.md has no mpc_input binding"
    return re.findall(r'\("(\w+)",', m.group(1))


def test_input_struct_layout(pkg):
    """The ctypes mpc_input (engine._Input) and INTEGRATION.md's minimal binding
    match the header as libmpc.so was compiled: size, field order, offsets."""
    e = pkg.engine
    L = e.lib()
    n = len(e._Input._fields_)
    off = (ctypes.c_size_t * n)()
    size = L.mpc_input_layout(off, n)
    assert size == ctypes.sizeof(e._Input)
    assert n == 24  # MPC_INPUT_FIELDS
    for k, (name, _) in enumerate(e._Input._fields_):
        assert off[k] == getattr(e._Input, name).offset, name
    assert _integration_fields() == [f for f, _ in e._Input._fields_]
    hdr = open(os.path.join(REPO, "include", "mpc.h")).read()
    body = re.sub(r"/\*.*?\*/", "", hdr[hdr.index("typedef struct {"):hdr.index("} mpc_input;")], flags=re.S)
    names = re.findall(r"^\s+[\w\s\*]+?\b(\w+);", body, re.M)
    assert names == [f for f, _ in e._Input._fields_]


def test_plan_info_no_overrides(pkg):
    """Product builds ignore the planners' measurement overrides:
    the env variables change nothing and mpc_plan_info reports none."""
    env = dict(os.environ, MPC_PARSE_GEOMETRY="2,1024,8", MPC_PARSE_WGS="3")
    code = ("import importlib,sys; sys.path.insert(0, %r); pkg = importlib.import_module('minion-plasmid-consensus_amd'); "
            "g = pkg.engine.geometry([2686, 2686], [100000, 100000], 63 << 20); "
            "print(g['overrides'], g['tally_mode'], g['parse_window'], g['parse_waves'], g['parse_workgroups'])" % REPO)
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, check=True).stdout.split()
    ref = pkg.engine.geometry([2686, 2686], [100000, 100000], 63 << 20)
    assert out == [str(x) for x in (0, ref["tally_mode"], ref["parse_window"], ref["parse_waves"], ref["parse_workgroups"])]


@pytest.mark.parametrize("order", ["lib_first", "torch_first"])
def test_one_hip_runtime_either_order(order):
    """libmpc.so and PyTorch share ONE HIP runtime whichever loads first
    (two runtimes in one process broke the first HIP call); the
    host-only planner does not import torch."""
    steps = {"lib_first": "e.lib(); g = e.geometry([2686], [1000], 1 << 20); t = 'torch' in sys.modules; import torch",
             "torch_first": "import torch; t = False; e.lib()"}[order]
    code = ("import importlib, sys; sys.path.insert(0, %r); e = importlib.import_module('minion-plasmid-consensus_amd.engine'); "
            "%s; print(len(e._hip_runtime_paths()), t)" % (REPO, steps))
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, check=True).stdout.split()
    assert out == ["1", "False"], out


def test_product_build_flags(pkg):
    """The shipped libmpc.so is the product build: no stamps, no planner
    overrides, no kernel variant macro (the timing ablations
    live in exp/ablations.patch, not in the product source)."""
    lib = pkg.engine.lib()
    lib.mpc_build_flags.restype = ctypes.c_int
    assert lib.mpc_build_flags() == 0
    src = open(os.path.join(REPO, "minion-plasmid-consensus_amd", "csrc", "mpc_kernels.hip")).read()
    assert "MPC_ABL_" not in src and "wrong results" not in src


def test_hip_runtime_soname_check(pkg, monkeypatch):
    """the torch-first preload compares SONAMEs.  Same SONAME ->
    map PyTorch's copy by path; a different one (PyTorch on another HIP major)
    -> MpcError naming both, raised before libmpc.so is loaded and without
    initialising any HIP runtime."""
    e = pkg.engine
    need = [x for x in e._elf_dynamic(e.LIB_PATH)[1] if x.startswith("libamdhip64.so")]
    assert len(need) == 1
    tpath = e._torch_hip_runtime()
    if tpath is not None:
        assert e._elf_dynamic(tpath)[0].startswith("libamdhip64.so")
    monkeypatch.setattr(e, "_torch_hip_runtime", lambda: "/x/libamdhip64.so")
    monkeypatch.setattr(e, "_elf_dynamic", lambda p: ("libamdhip64.so.9", []) if p.startswith("/x/")
                        else (None, ["libamdhip64.so.7"]))
    monkeypatch.setattr(e, "_torch", lambda: pytest.fail("torch must not be touched"))
    monkeypatch.setattr(e.ctypes, "CDLL", lambda *a, **k: pytest.fail("nothing may be loaded"))
    with pytest.raises(e.MpcError) as err:
        e._preload_hip_runtime()
    assert "libamdhip64.so.9" in str(err.value) and "libamdhip64.so.7" in str(err.value)


def test_elf_dynamic_reads_ranges(tmp_path):
    """_elf_dynamic parses the real libraries and rejects a truncated file."""
    import importlib
    e = importlib.import_module("minion-plasmid-consensus_amd.engine")
    so, need = e._elf_dynamic(e.LIB_PATH)
    assert any(x.startswith("libamdhip64.so") for x in need)
    cut = tmp_path / "cut.so"
    cut.write_bytes(open(e.LIB_PATH, "rb").read(200))
    assert e._elf_dynamic(str(cut)) == (None, [])
