#!/usr/bin/env python3
"""Experiment builds: patch a COPY of csrc/mpc_kernels.hip (string replacements),
compile to exp/v/<name>.so.  Never imported by the product; timing only.
  python3 exp/mkvar.py name=patchset [name=patchset ...]   (patch sets in exp/patches.py)"""
import os, subprocess, sys, importlib.util
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(R, "minion-plasmid-consensus_amd", "csrc", "mpc_kernels.hip")
spec = importlib.util.spec_from_file_location("patches", os.path.join(R, "exp", "patches.py"))
P = importlib.util.module_from_spec(spec); spec.loader.exec_module(P)
os.makedirs(os.path.join(R, "exp", "v"), exist_ok=True)
procs = []
for arg in sys.argv[1:]:
    name, sets = arg.split("=") if "=" in arg else (arg, arg)
    s = open(SRC).read()
    flags = []
    for ps in sets.split("+"):
        if ps == "base": continue
        flags += getattr(P, "FLAGS", {}).get(ps, [])
        for old, new in P.PATCHES[ps]:
            assert s.count(old) == 1, (ps, old[:80], s.count(old))
            s = s.replace(old, new)
    tu = os.path.join(R, "exp", "v", name + ".hip")
    open(tu, "w").write(s)
    so = os.path.join(R, "exp", "v", name + ".so")
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-I", os.path.join(R, "include"), "-I", os.path.join(R, "minion-plasmid-consensus_amd", "csrc"), "-o", so, tu] + flags
    procs.append((name, subprocess.Popen(cmd)))
for name, p in procs:
    print(name, "ok" if p.wait() == 0 else "FAILED")
