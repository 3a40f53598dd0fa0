#!/usr/bin/env python3
"""Time the parse phase ALONE (K_clear + K_parse, HIP events) of library
variants; later phases never run, so experiment builds that skip stores are
safe.   KEXP_CFG=c1..c5 (bench.py workloads) python3 scripts/kparse_only.py lib1.so [lib2.so ...]"""
import os, subprocess, sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = os.path.join(REPO, "scripts", "kp_child.py")
for lib in sys.argv[1:]:
    env = dict(os.environ, KEXP_LIB=os.path.abspath(lib))
    p = subprocess.run([sys.executable, CHILD], env=env, capture_output=True, text=True, timeout=300)
    line = [l for l in p.stdout.splitlines() if l.startswith("KP")]
    print(os.path.basename(lib), line[0][3:] if line else ("FAILED rc=%d %s" % (p.returncode, p.stderr[-800:])), flush=True)
