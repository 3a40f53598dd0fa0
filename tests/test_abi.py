"""The C-ABI library loads and exports every function declared in include/mpc.h
(no compute calls: runs without a GPU)."""
import ctypes
import os
import re

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared(header="mpc.h"):
    txt = open(os.path.join(REPO, "include", header)).read()
    return sorted(set(re.findall(r"^(?:int|void|const char\*)\s+(mpc_\w+)\(", txt, re.M)))


def test_header_declares_entry_points():
    names = declared()
    for f in ("mpc_version", "mpc_plan_create", "mpc_plan_bind", "mpc_parse", "mpc_index", "mpc_runs", "mpc_tally",
              "mpc_layout", "mpc_rows", "mpc_consensus", "mpc_run", "mpc_profile_kernel"):
        assert f in names


def test_library_exports_all(pkg):
    path = pkg._build.build_hip()
    lib = ctypes.CDLL(path)
    for name in declared():
        assert hasattr(lib, name), name
    lib.mpc_version.restype = ctypes.c_int
    assert lib.mpc_version() == pkg.engine.ABI_VERSION == 4


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
