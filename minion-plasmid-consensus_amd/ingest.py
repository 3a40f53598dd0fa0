"""Host ingest: Steps 1-3 of /root/reference/src/mapped_paf_read_parser.py.

Produces the packed per-read arrays the device path consumes.  The semantics
follow the reference line by line (text mode with universal newlines, str
rstrip/upper/split, Python int(), first alignment per read name wins, whole
header line as the read name, Python slicing for the flanks); where the
reference raises, this raises :class:`IngestError` (the CLI then exits 1 and
writes nothing, like the reference).

  Step 1  reference FASTA       :161-184  -> read_reference()
  Step 2  PAF                   :192-245  -> read_paf()
  Step 3  reads FASTA + flanks  :253-277  -> read_flanks()

``pack_sample`` uses the native parser (libmpc_ingest.so, include/mpc_ingest.h:
memory-mapped, multi-threaded, same results) and falls back to the Python
restatement below when the native library declines an input feature it does
not restate (non-ASCII bytes, carriage returns, integers in a form only
Python's int() accepts) or is not built.  Non-ASCII text is transcoded to one
byte per character with the same semantics (transcode_*: the device path is
byte-based).
"""
import ctypes
import os

import numpy as np

BASE_COMPLIMENT = {"A": "T", "T": "A", "G": "C", "C": "G", "N": "N"}  # :27
# lowest target start the device takes (mpc.h MPC_TSTART_MIN: -2^28)
TSTART_MIN = -(1 << 28)
_RC_TABLE = str.maketrans("ACGTN", "TGCAN")
_ALLOWED_RC = frozenset("ACGTN")


class IngestError(Exception):
    """An input the reference rejects (it would raise and exit with status 1)."""


def read_reference(path):
    """Concatenate every non-header line, rstrip()ed and upper-cased (:161-165)."""
    parts = []
    with open(path, "r") as fh:
        for line in fh:
            if not line.startswith(">"):
                parts.append(line.rstrip().upper())
    return "".join(parts)


def read_paf(path):
    """First alignment per read name (:237-243), in first-occurrence order.

    Returns (records, n_lines); each record is [name, qs', qe', tstart, strand, cs].
    """
    recs = {}
    n_lines = 0
    with open(path, "r") as fh:
        for line in fh:
            f = line.rstrip().split("\t")
            n_lines += 1
            try:
                name = f[0]
                qlen = int(f[1])
                qs = int(f[2])
                qe = int(f[3])
                ts = int(f[7])
                strand = f[4]
            except (IndexError, ValueError) as e:
                raise IngestError(f"PAF line {n_lines}: {type(e).__name__}: {e}") from None
            if strand == "-":
                qs, qe = qlen - qe, qlen - int(f[2])  # :226-228
            cs = None
            for e in f:  # first field starting with "cs:" (:231)
                if e.startswith("cs:"):
                    cs = e[3:]
                    break
            if cs is None:
                raise IngestError(f"PAF line {n_lines}: IndexError: no cs: tag")
            if name not in recs:
                recs[name] = [name, qs, qe, ts, strand, cs]
    return list(recs.values()), n_lines


def read_flanks(path, recs):
    """Upstream / downstream flanks of every PAF read (:253-277).

    Only records named in the PAF are materialized: for the others the
    reference only runs rstrip()/upper(), which cannot fail.  A duplicate FASTA
    name is processed again and the last one wins.
    """
    by_name = {r[0]: r for r in recs}
    flanks = {}
    name = ""
    seq_parts = None

    def finish(name, parts):
        r = by_name.get(name)
        if name == "" or r is None:
            return
        seq = "".join(parts)
        if r[4] == "-":
            bad = set(seq) - _ALLOWED_RC
            if bad:
                raise IngestError(f"KeyError: {sorted(bad)[0]!r} (reverse complement of read {name})")
            seq = seq[::-1].translate(_RC_TABLE)
        flanks[name] = (seq[: r[1]], seq[r[2]:])

    with open(path, "r") as fh:
        for line in fh:
            if line.startswith(">"):
                if seq_parts is not None:
                    finish(name, seq_parts)
                name = line.rstrip()[1:]
                seq_parts = [] if name in by_name else None
            elif seq_parts is not None:
                seq_parts.append(line.rstrip().upper())
    if seq_parts is not None:
        finish(name, seq_parts)
    return flanks


# Non-ASCII text (the reference decodes its files as str, :163, :196, :257):
# the device path works on bytes, one byte per character, so every non-ASCII
# character is transcoded to ONE byte with the same effect on the reference's
# semantics.  A character the reference would write as a base ({A,T,C,G} dict
# keys after .upper(), :59-61 / :70-71 / :87 / :96) and that is not one of them
# becomes NON_BASE (a byte outside ACGT, so the device raises the same KeyError
# if and only if it is written); coordinates count characters, as str does.
NON_BASE = 0x80
_SPECIAL = ":Z+-*"  # SPECIAL_CHARS (:290)


def _base_byte(c):
    """One byte for character c where only its .upper() as a base matters."""
    if ord(c) < 128:
        return c.encode("ascii")
    u = c.upper()
    return u.encode("ascii") if u in ("A", "C", "G", "T") else bytes((NON_BASE,))


def transcode_ref(refseq):
    """The upper-cased reference string (:165) -> one byte per character."""
    try:
        return refseq.encode("ascii")
    except UnicodeEncodeError:
        return b"".join(_base_byte(c) for c in refseq)


def transcode_flank(seq):
    """An upper-cased flank (:264-265, :270) -> one byte per character: every
    flank character is written as a base (:303, :323)."""
    try:
        return seq.encode("ascii")
    except UnicodeEncodeError:
        return b"".join(_base_byte(c) for c in seq)


def transcode_cs(cs):
    """A cs tag -> ASCII bytes with the same tokens (:306-320) and the same
    effect of every operation (:74-104): a ':' operand that holds non-ASCII
    characters is replaced by the value Python's int() gives it (Unicode
    digits and spaces; a negative value matches nothing, like 0; a ValueError
    stays one), '-' and 'Z' operands keep their length in characters, '*' and
    '+' operand characters map through _base_byte."""
    try:
        return cs.encode("ascii")
    except UnicodeEncodeError:
        pass
    out, k, n = [], 0, len(cs)
    while k < n:
        j = k + 1 if cs[k] in _SPECIAL else k  # operator (or none: "Unknown operator", :100)
        e = j
        while e < n and cs[e] not in _SPECIAL:
            e += 1
        op, operand = cs[k:j], cs[j:e]
        if op == ":" and operand and not operand.isascii():
            try:
                v = int(operand)
                operand = str(v) if v > 0 else "0"
            except ValueError:
                operand = "x"  # int() fails on the device too
        elif op in (":", "-", "Z", ""):
            operand = "".join(c if ord(c) < 128 else "n" for c in operand)
        out.append(op.encode("ascii"))
        out.append(b"".join(_base_byte(c) for c in operand) if op in ("*", "+") else operand.encode("ascii"))
        k = e
    return b"".join(out)


def _concat(items):
    off = np.zeros(len(items) + 1, dtype=np.int64)
    if items:
        np.cumsum(np.fromiter((len(x) for x in items), dtype=np.int64, count=len(items)), out=off[1:])
    return b"".join(items), off


class _IngestOut(ctypes.Structure):
    _fields_ = [
        ("ref", ctypes.POINTER(ctypes.c_uint8)), ("ref_len", ctypes.c_int64),
        ("cs", ctypes.POINTER(ctypes.c_uint8)), ("cs_off", ctypes.POINTER(ctypes.c_int64)),
        ("tstart", ctypes.POINTER(ctypes.c_int64)),
        ("up", ctypes.POINTER(ctypes.c_uint8)), ("up_off", ctypes.POINTER(ctypes.c_int64)),
        ("down", ctypes.POINTER(ctypes.c_uint8)), ("down_off", ctypes.POINTER(ctypes.c_int64)),
        ("aligned", ctypes.POINTER(ctypes.c_int64)),
        ("n_reads", ctypes.c_int64), ("n_alignments", ctypes.c_int64),
        ("status", ctypes.c_int32), ("message", ctypes.c_char * 256),
    ]


INGEST_OK, INGEST_ERROR, INGEST_FALLBACK = 0, 1, 2
INGEST_ABI = 3  # mpc_ingest_version() of the library these bindings expect
_ingest_lib = None


def _native():
    global _ingest_lib
    if _ingest_lib is None:
        from . import _build
        path = _build.LIBINGEST
        try:
            _build.build_ingest()  # no-op unless missing or older than its sources
        except Exception:  # no compiler: a present library is still used, else the Python ingest
            if not os.path.exists(path):
                _ingest_lib = False
                return None
        L = ctypes.CDLL(path)
        L.mpc_ingest_version.restype = ctypes.c_int
        if L.mpc_ingest_version() != INGEST_ABI:
            raise IngestError(f"{path}: ABI {L.mpc_ingest_version()} != {INGEST_ABI} (stale build: "
                              "rebuild with __graft_entry__.build())")
        L.mpc_ingest.restype = ctypes.c_int
        L.mpc_ingest.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int,
                                 ctypes.POINTER(_IngestOut)]
        L.mpc_ingest_multi.restype = ctypes.c_int
        L.mpc_ingest_multi.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_char_p),
                                       ctypes.c_char_p, ctypes.c_int, ctypes.POINTER(_IngestOut)]
        L.mpc_ingest_free.argtypes = [ctypes.POINTER(_IngestOut)]
        L.mpc_write_calls.restype = ctypes.c_int
        L.mpc_write_calls.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_char_p, ctypes.c_char_p,
                                      ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_int]
        L.mpc_py_float_repr.restype = ctypes.c_int
        L.mpc_py_float_repr.argtypes = [ctypes.c_double, ctypes.c_char_p, ctypes.c_int]
        _ingest_lib = L
    return _ingest_lib or None


def pack_sample_native(ref_path, paf_path, reads_path, n_threads=0):
    """Steps 1-3 through libmpc_ingest.so.  Returns the packed dict, None when the
    native parser declines the input (use :func:`pack_sample_python`), or raises
    :class:`IngestError` where the reference raises."""
    r = pack_samples_native([(ref_path, paf_path)], reads_path, n_threads)
    if r is None:
        return None
    if isinstance(r[0], IngestError):
        raise r[0]
    return r[0]


def pack_samples_native(jobs, reads_path, n_threads=0):
    """Steps 1-3 of several (ref_path, paf_path) jobs against ONE reads FASTA,
    scanned once (mpc_ingest_multi).  Returns None when the library is missing,
    else a list with, per job, the packed dict, None (declined: use the Python
    ingest) or the :class:`IngestError` the reference raises for that job."""
    L = _native()
    if L is None:
        return None
    nj = len(jobs)
    enc = lambda p: os.fsencode(p)
    refs = (ctypes.c_char_p * nj)(*[enc(r) for r, _ in jobs])
    pafs = (ctypes.c_char_p * nj)(*[enc(p) for _, p in jobs])
    outs = (_IngestOut * nj)()
    L.mpc_ingest_multi(nj, refs, pafs, enc(reads_path), int(n_threads), outs)
    res = []
    for j in range(nj):
        own = _IngestBuffers(L, outs, j)
        o = own.out
        if o.status == INGEST_FALLBACK:
            res.append(None)
        elif o.status != INGEST_OK:
            res.append(IngestError(o.message.decode(errors="replace")))
        else:
            res.append(_views(own))
    return res


def _views(own):
    o = own.out
    n = o.n_reads
    # zero-copy: the arrays are views of the library's buffers (a GB of cs at
    # C3), freed once the last view is gone
    cs_off = own.view(o.cs_off, n + 1, ctypes.c_int64)
    up_off = own.view(o.up_off, n + 1, ctypes.c_int64)
    dn_off = own.view(o.down_off, n + 1, ctypes.c_int64)
    return dict(
        ref=own.view(o.ref, o.ref_len, ctypes.c_uint8),
        cs=own.view(o.cs, int(cs_off[-1]), ctypes.c_uint8), cs_off=cs_off,
        tstart=own.view(o.tstart, n, ctypes.c_int64),
        up=own.view(o.up, int(up_off[-1]), ctypes.c_uint8), up_off=up_off,
        down=own.view(o.down, int(dn_off[-1]), ctypes.c_uint8), down_off=dn_off,
        aligned=own.view(o.aligned, n, ctypes.c_int64),
        n_alignments=int(o.n_alignments),
    )


class _IngestBuffers:
    """Owner of one mpc_ingest result (element j of an output array): numpy views
    of its buffers keep it alive (through their ctypes base), and it frees them
    when the last view goes."""

    def __init__(self, lib, outs, j):
        self.lib = lib
        self.outs = outs  # keeps the array alive
        self.out = outs[j]

    def view(self, ptr, k, ct):
        if k <= 0:
            return np.zeros(0, dtype=ct)
        buf = (ct * int(k)).from_address(ctypes.addressof(ptr.contents))
        buf._owner = self
        return np.frombuffer(buf, dtype=ct)

    def __del__(self):
        lib = getattr(self, "lib", None)
        if lib is not None:
            lib.mpc_ingest_free(ctypes.byref(self.out))
            self.lib = None


def pack_sample(ref_path, paf_path, reads_path, native=True):
    """Steps 1-3 for one (assembly, PAF) sample -> dict of packed numpy arrays
    (native parser when it accepts the input, else the Python restatement)."""
    if native:
        r = pack_sample_native(ref_path, paf_path, reads_path)
        if r is not None:
            return r
    return pack_sample_python(ref_path, paf_path, reads_path)


def job_groups(jobs):
    """Indices of (ref_path, paf_path, reads_path) jobs grouped by reads file, each
    group in job order, groups in the order of their first job."""
    groups = {}
    for j, (_, _, reads) in enumerate(jobs):
        groups.setdefault(os.fspath(reads), []).append(j)
    return list(groups.values())


def pack_group(jobs, native=True):
    """Steps 1-3 for jobs that share ONE reads file (one scan of it) -> per job,
    its packed dict or the :class:`IngestError` the reference raises for it
    (not raised here); jobs the native parser declines take the Python path."""
    out = [None] * len(jobs)
    if native and jobs:
        r = pack_samples_native([(ref, paf) for ref, paf, _ in jobs], jobs[0][2])
        if r is not None:
            out = list(r)
    for j, (ref, paf, reads) in enumerate(jobs):
        if out[j] is None:
            try:
                out[j] = pack_sample_python(ref, paf, reads)
            except (IngestError, UnicodeDecodeError, OSError) as e:
                out[j] = e
    return out


def pack_samples(jobs, native=True):
    """Steps 1-3 for (ref_path, paf_path, reads_path) jobs -> list of packed
    dicts, in job order.  Jobs sharing a reads file are ingested together (one
    scan of it); a job the native parser declines takes the Python path.  The
    first job (in order) the reference would reject raises its IngestError."""
    out = [None] * len(jobs)
    if native:
        groups = {}
        for j, (_, _, reads) in enumerate(jobs):
            groups.setdefault(os.fspath(reads), []).append(j)
        for reads, idx in groups.items():
            r = pack_samples_native([(jobs[j][0], jobs[j][1]) for j in idx], reads)
            if r is not None:
                for j, x in zip(idx, r):
                    out[j] = x
    for j, (ref, paf, reads) in enumerate(jobs):
        if isinstance(out[j], IngestError):
            raise out[j]
        if out[j] is None:
            out[j] = pack_sample_python(ref, paf, reads)
    return out


def pack_sample_python(ref_path, paf_path, reads_path):
    """Steps 1-3 for one (assembly, PAF) sample in Python -> dict of packed numpy arrays."""
    refseq = read_reference(ref_path)
    recs, n_lines = read_paf(paf_path)
    flanks = read_flanks(reads_path, recs)
    cs, up, down, ts, aligned = [], [], [], [], []
    for name, qs, qe, t, strand, c in recs:
        fl = flanks.get(name)
        if fl is None:  # paf[read_name]["upstream_seq"] -> KeyError (:303)
            raise IngestError(f"KeyError: 'upstream_seq' (read {name} not in {reads_path})")
        if t < TSTART_MIN or t >= 2 ** 31:  # (negative starts: the device wraps them like Python, mpc.h)
            raise IngestError(f"target start {t} of read {name} out of range (unsupported)")
        cs.append(transcode_cs(c))
        up.append(transcode_flank(fl[0]))
        down.append(transcode_flank(fl[1]))
        ts.append(t)
        aligned.append(qe - qs)
    cs_b, cs_off = _concat(cs)
    up_b, up_off = _concat(up)
    dn_b, dn_off = _concat(down)
    return dict(
        ref=np.frombuffer(transcode_ref(refseq), dtype=np.uint8),
        cs=np.frombuffer(cs_b, dtype=np.uint8), cs_off=cs_off,
        tstart=np.asarray(ts, dtype=np.int64),
        up=np.frombuffer(up_b, dtype=np.uint8), up_off=up_off,
        down=np.frombuffer(dn_b, dtype=np.uint8), down_off=dn_off,
        aligned=np.asarray(aligned, dtype=np.int64),
        n_alignments=n_lines,
    )
