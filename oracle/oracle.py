"""CPU oracle for the pileup + consensus path -- TEST INFRASTRUCTURE ONLY.

Only tests/, ``__graft_entry__.smoke()`` and bench.py's ``cpu_baseline`` leg may
import this module.  The product package never imports it (the HIP path fails
loudly instead of falling back to anything here).

``run_packed`` drives ``mpc_oracle.c`` (a step-for-step restatement of
/root/reference/src/mapped_paf_read_parser.py:37-104, :285-439) on the packed
per-read inputs; ``format_outputs`` restates the writers (:446-463);
``ingest_files`` restates Steps 1-3 (:161-277) in pure Python so whole-file
cases can be replayed without the reference.  Parity of this oracle with the
reference itself is pinned by tests/test_oracle_golden.py against
tests/golden/ (outputs of the reference script, scripts/make_golden.py).
"""
import ctypes
import os
import subprocess

import re

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libmpc_oracle.so")

ERR_NAMES = {0: "ok", 1: "KeyError", 2: "IndexError", 3: "ValueError", 4: "UnknownOperator", 5: "NoMemory"}


class _Out(ctypes.Structure):
    _fields_ = [
        ("n_calls", ctypes.c_int64),
        ("base", ctypes.POINTER(ctypes.c_char)),
        ("chrom1", ctypes.POINTER(ctypes.c_char)),
        ("chrom2", ctypes.POINTER(ctypes.c_char)),
        ("count", ctypes.POINTER(ctypes.c_int64)),
        ("count2", ctypes.POINTER(ctypes.c_int64)),
        ("total", ctypes.POINTER(ctypes.c_int64)),
        ("xpos", ctypes.POINTER(ctypes.c_int64)),
        ("slot", ctypes.POINTER(ctypes.c_int64)),
        ("max_depth", ctypes.c_int64),
        ("err", ctypes.c_int),
        ("err_read", ctypes.c_int64),
    ]


_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH) or os.path.getmtime(LIB_PATH) < os.path.getmtime(
            os.path.join(HERE, "mpc_oracle.c")
        ):
            build()
        L = ctypes.CDLL(LIB_PATH)
        L.mpc_oracle_run.restype = ctypes.c_int
        L.mpc_oracle_run.argtypes = [ctypes.c_char_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p,
                                     ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                     ctypes.c_void_p, ctypes.c_void_p, ctypes.c_double, ctypes.c_double,
                                     ctypes.POINTER(_Out)]
        L.mpc_oracle_free.argtypes = [ctypes.POINTER(_Out)]
        _lib = L
    return _lib


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def run_packed(ref, cs, cs_off, tstart, up, up_off, down, down_off, mdf, gtf):
    """Pileup + consensus for one sample.  Byte buffers are numpy uint8 / bytes,
    offsets int64 (N+1).  Returns a dict of numpy arrays (one entry per emitted
    slot, in output order) or raises OracleError."""
    ref = bytes(ref)
    cs = np.ascontiguousarray(np.frombuffer(bytes(cs), dtype=np.uint8) if not isinstance(cs, np.ndarray) else cs, dtype=np.uint8)
    up = np.ascontiguousarray(np.frombuffer(bytes(up), dtype=np.uint8) if not isinstance(up, np.ndarray) else up, dtype=np.uint8)
    down = np.ascontiguousarray(np.frombuffer(bytes(down), dtype=np.uint8) if not isinstance(down, np.ndarray) else down, dtype=np.uint8)
    cs_off = np.ascontiguousarray(cs_off, dtype=np.int64)
    up_off = np.ascontiguousarray(up_off, dtype=np.int64)
    down_off = np.ascontiguousarray(down_off, dtype=np.int64)
    tstart = np.ascontiguousarray(tstart, dtype=np.int64)
    n_reads = len(tstart)
    # keep non-empty buffers alive for ctypes
    cs_b = cs if cs.size else np.zeros(1, np.uint8)
    up_b = up if up.size else np.zeros(1, np.uint8)
    dn_b = down if down.size else np.zeros(1, np.uint8)
    ts_b = tstart if tstart.size else np.zeros(1, np.int64)
    out = _Out()
    L = lib()
    L.mpc_oracle_run(ref, len(ref), n_reads, _ptr(cs_b), _ptr(cs_off), _ptr(ts_b), _ptr(up_b), _ptr(up_off),
                     _ptr(dn_b), _ptr(down_off), float(mdf), float(gtf), ctypes.byref(out))
    try:
        if out.err:
            raise OracleError(out.err, out.err_read)
        k = out.n_calls

        def arr(p, dt):
            if k == 0:
                return np.zeros(0, dtype=dt)
            return np.ctypeslib.as_array(p, shape=(k,)).copy()

        def chars(p):
            if k == 0:
                return np.zeros(0, dtype=np.uint8)
            return np.frombuffer(ctypes.string_at(p, k), dtype=np.uint8).copy()

        res = {
            "base": chars(out.base),
            "chrom1": chars(out.chrom1),
            "chrom2": chars(out.chrom2),
            "count": arr(out.count, np.int64),
            "count2": arr(out.count2, np.int64),
            "total": arr(out.total, np.int64),
            "xpos": arr(out.xpos, np.int64),
            "slot": arr(out.slot, np.int64),
            "max_depth": int(out.max_depth),
        }
    finally:
        L.mpc_oracle_free(ctypes.byref(out))
    return res


class OracleError(Exception):
    def __init__(self, code, read):
        super().__init__(f"{ERR_NAMES.get(code, code)} (read {read})")
        self.code = code
        self.read = read


def format_outputs(res):
    """Writers of the reference (:446-463): returns (consensus, chromat, accuracies) text."""
    base = bytes(res["base"]).decode("ascii")
    c1 = bytes(res["chrom1"]).decode("ascii")
    c2 = bytes(res["chrom2"]).decode("ascii")
    cons = ">consensus\n" + base + "\n"
    lines = ["pos\tbase\tcount\n"]
    acc = ["pos\taccuracy\n"]
    cnt, cnt2, tot = res["count"].tolist(), res["count2"].tolist(), res["total"].tolist()
    for i in range(len(base)):
        lines.append("%d\t%s\t%d\n" % (i + 1, c1[i], cnt[i]))
        lines.append("%d\t%s\t%d\n" % (i + 1, c2[i], cnt2[i]))
        acc.append("{}\t{}\n".format(i + 1, 100 * (cnt[i] / tot[i])))
    return cons, "".join(lines), "".join(acc)


BASE_COMPLIMENT = {"A": "T", "T": "A", "G": "C", "C": "G", "N": "N"}


_ACGT = frozenset("ACGT")


def _base_bytes(s):
    """One byte per character of a str whose characters are only ever used as
    bases (reference :184, flanks :303/:323): a non-ASCII character whose
    .upper() is not a single A/C/G/T can never be a dict key -> 0x80."""
    return bytes(ord(c) if ord(c) < 128 else (ord(c.upper()) if c.upper() in _ACGT else 0x80) for c in s)


def _cs_bytes(cs):
    """A cs tag -> bytes, one operation at a time (:306-320): ':' operands by
    their int() value (Unicode digits; ValueError kept as one), '-' and 'Z'
    operands by their length in characters, '*' / '+' operands as bases."""
    if cs.isascii():
        return cs.encode("ascii")
    out = bytearray()
    for op, operand in re.findall(r"([:Z+*-]?)([^:Z+*-]*)", cs):
        out += op.encode("ascii")
        if op == ":" and not operand.isascii():
            try:
                out += b"%d" % max(int(operand), 0)
            except ValueError:
                out += b"?"
        elif op in ("*", "+"):
            out += _base_bytes(operand)
        else:
            out += b"n" * len(operand) if not operand.isascii() else operand.encode("ascii")
    return bytes(out)


def ingest_files(ref_path, paf_path, reads_path):
    """Pure-Python restatement of Steps 1-3 (:161-277).  Returns the packed
    inputs of one sample, or raises KeyError/IndexError/ValueError exactly where
    the reference would (a PAF read missing from the FASTA raises KeyError)."""
    refseq = ""
    for line in open(ref_path, "r"):
        if not line.startswith(">"):
            refseq += line.rstrip().upper()
    paf = {}
    for line in open(paf_path, "r"):
        f = line.rstrip().split("\t")
        name = f[0]
        qlen = int(f[1])
        qs = int(f[2])
        qe = int(f[3])
        ts = int(f[7])
        strand = f[4]
        if strand == "-":
            qs = qlen - qe
            qe = qlen - int(f[2])
        cstag = [e for e in f if e.startswith("cs:")][0][3:]
        if name not in paf:
            paf[name] = {"qs": qs, "qe": qe, "ts": ts, "strand": strand, "cs": cstag}
    name = ""
    seq = ""

    def finish(name, seq):
        if name != "" and name in paf:
            if paf[name]["strand"] == "-":
                seq = "".join([BASE_COMPLIMENT[x.upper()] for x in seq[::-1]])
            paf[name]["up"] = seq[: paf[name]["qs"]]
            paf[name]["down"] = seq[paf[name]["qe"]:]

    for line in open(reads_path, "r"):
        if line.startswith(">"):
            finish(name, seq)
            name = line.rstrip()[1:]
            seq = ""
        else:
            seq += line.rstrip().upper()
    finish(name, seq)
    recs = list(paf.values())
    for r in recs:
        if "up" not in r:
            raise KeyError("upstream_seq")
    cs = [_cs_bytes(r["cs"]) for r in recs]
    up = [_base_bytes(r["up"]) for r in recs]
    dn = [_base_bytes(r["down"]) for r in recs]
    off = lambda xs: np.concatenate([[0], np.cumsum([len(x) for x in xs], dtype=np.int64)]).astype(np.int64)
    return dict(ref=_base_bytes(refseq), cs=b"".join(cs), cs_off=off(cs), tstart=np.array([r["ts"] for r in recs], np.int64),
                up=b"".join(up), up_off=off(up), down=b"".join(dn), down_off=off(dn))
