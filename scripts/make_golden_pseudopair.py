#!/usr/bin/env python3
"""Generate tests/golden_pseudopair/ by running the REFERENCE src/pseudopair_reads.py
(build container only, ``python3 -B``: nothing is written into the reference tree).

Each case holds in.paf (gzip'd when > 4 KB) and, per --min_align_length run,
the reference's exit status and its output file (absent when it failed before
opening it)."""
import gzip
import json
import os
import random
import shutil
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(REPO, "tests", "golden_pseudopair")
SCRIPT = "/root/reference/src/pseudopair_reads.py"


def line(name, qlen, qs, qe, strand, extra=True):
    f = [name, str(qlen), str(qs), str(qe), strand]
    if extra:
        f += ["tig", "5000", "0", str(qe - qs), str(qe - qs), str(qe - qs), "60", "tp:A:P"]
    return "\t".join(f) + "\n"


def synthetic(seed, n, dup_frac=0.2):
    rng = random.Random(seed)
    out = []
    names = ["read_%d" % k for k in range(n)]
    for nm in names:
        reps = 1
        u = rng.random()
        if u < dup_frac:
            reps = rng.choice([2, 2, 3, 4])
        for _ in range(reps):
            qlen = rng.randint(500, 20000)
            qs = rng.randint(0, 200)
            qe = rng.randint(qs, qlen)
            out.append((rng.random(), line(nm, qlen, qs, qe, rng.choice("++-"))))
    out.sort()  # interleave duplicates through the file
    return "".join(x for _, x in out)


CASES = {
    "basic": ("".join([line("a", 1000, 10, 900, "+"), line("b", 800, 0, 700, "-"), line("c", 900, 5, 100, "+"),
                       line("a", 1000, 0, 1000, "-"), line("d", 700, 0, 600, "-"), line("e", 500, 0, 450, "+"),
                       line("a", 1000, 0, 500, "-"), line("f", 400, 0, 400, "+"), line("b", 800, 0, 800, "+"),
                       line("b", 800, 0, 800, "-"), line("b", 800, 0, 10, "+")]), [0, 100, 450, 890, 10 ** 6]),
    "empty": ("", [100, None]),
    "five_fields": (line("x", 100, 0, 90, "+", False) + line("y", 100, 0, 90, "-", False)
                    + line("z", 100, 0, 90, "+", False).rstrip("\n"), [0]),
    "strand_other": (line("p", 100, 0, 90, ".") + line("q", 100, 0, 90, "+") + line("r", 100, 0, 90, "*"), [0]),
    "short_line": (line("a", 100, 0, 90, "+") + "b\t100\t0\n", [0]),
    "bad_int": (line("a", 100, 0, 90, "+") + "b\tx\t0\t90\t+\n", [0]),
    "min_missing": (line("a", 100, 0, 90, "+"), [None]),
    "py_int_forms": ("a\t 100\t+0\t90\t+\tt\n" + "b\t1_00\t0\t9_0\t-\tt\n" + "c\t100\t 0 \t90\t-\tt\n", [0, 91]),
    "crlf": (line("a", 100, 0, 90, "+").replace("\n", "\r\n") + line("b", 100, 0, 90, "-").replace("\n", "\r\n"),
             [0]),
    "blank_line_end": (line("a", 100, 0, 90, "+") + line("b", 100, 0, 90, "-") + "\n", [0]),
    "negative_len": (line("a", 100, 90, 10, "+") + line("b", 100, 0, 90, "-"), [-100, 0]),
    "synthetic_2k": (synthetic(5, 2000), [0, 5000, 12000]),
    "synthetic_20k": (synthetic(6, 20000, 0.35), [1000]),
}


def wfile(path, data):
    data = data.encode() if isinstance(data, str) else data
    if len(data) > 4096:
        with open(path + ".gz", "wb") as raw:
            with gzip.GzipFile(fileobj=raw, mode="wb", compresslevel=9, mtime=0, filename="") as f:
                f.write(data)
    else:
        with open(path, "wb") as f:
            f.write(data)


def main():
    os.makedirs(OUT, exist_ok=True)
    env = dict(os.environ, PYTHONDONTWRITEBYTECODE="1")
    for name, (paf, mins) in CASES.items():
        cdir = os.path.join(OUT, name)
        if os.path.exists(cdir):
            shutil.rmtree(cdir)
        os.makedirs(cdir)
        wfile(os.path.join(cdir, "in.paf"), paf)
        runs = []
        with tempfile.TemporaryDirectory() as tmp:
            pp = os.path.join(tmp, "in.paf")
            with open(pp, "w", newline="") as f:
                f.write(paf)
            for k, m in enumerate(mins):
                out = os.path.join(tmp, "pairs.txt")
                if os.path.exists(out):
                    os.remove(out)
                cmd = [sys.executable, "-B", SCRIPT, "--paf", pp, "--pseudopairs", out]
                if m is not None:
                    cmd += ["--min_align_length", str(m)]
                r = subprocess.run(cmd, env=env, capture_output=True, text=True)
                ent = {"min_align_length": m, "exit": r.returncode, "file": None}
                if os.path.exists(out):
                    ent["file"] = "run%d_pairs.txt" % k
                    wfile(os.path.join(cdir, ent["file"]), open(out, "rb").read())
                runs.append(ent)
        with open(os.path.join(cdir, "case.json"), "w") as f:
            json.dump({"runs": runs}, f, indent=1)
        print(name, [(r["min_align_length"], r["exit"], r["file"] is not None) for r in runs])


if __name__ == "__main__":
    main()
