"""ctypes binding of libmpc.so (include/mpc.h) + device buffer management.

PyTorch-ROCm is only the allocator/stream provider here: every input and the
single workspace are torch uint8 tensors on the GPU, and the C-ABI receives
raw device pointers.  There is no CPU fallback: if libmpc.so or a HIP device
is missing, :class:`Engine` raises.
"""
import ctypes
import os
import warnings

import numpy as np

from . import _build

LIB_PATH = _build.LIBMPC

ABI_VERSION = 9
MPC_ST_FLAGS, MPC_ST_FIRST_READ, MPC_ST_ROWS_NEEDED, MPC_ST_MIXED, MPC_ST_RSORT_PATH = 0, 1, 2, 3, 5
MPC_ST_WRAP_EVENTS, MPC_ST_WRAP_POS = 6, 7
DE_OP, DE_VALUE, DE_INDEX, DE_KEY, DE_CAPACITY, DE_INTERNAL, DE_UNSUPPORTED = 1, 2, 4, 8, 16, 32, 64
(BUF_STATUS, BUF_CALLS, BUF_NCALLS, BUF_MAXDEPTH, BUF_ROWS, BUF_ROWMETA, BUF_RIGHT_CNT, BUF_RIGHT_CNT_ALL,
 BUF_HASLEFT, BUF_MAXR, BUF_RUN_M, BUF_RUN_R, BUF_DIFF, BUF_SUB) = range(14)
PHASES = ("parse", "index", "runs", "tally", "layout", "rows")

DE_NAMES = {DE_OP: "Unknown operator", DE_VALUE: "ValueError", DE_INDEX: "IndexError", DE_KEY: "KeyError",
            DE_CAPACITY: "row capacity", DE_INTERNAL: "internal invariant",
            DE_UNSUPPORTED: "unsupported input (a negative target start the plan was not sized for, or an "
                            "advance of 2^22 or more from a negative coordinate)"}
K_PARSE, K_ODD, K_LEFT, K_FLANK, K_INS, K_RSORT = 0, 1, 2, 3, 4, 5
CS_PAD = 2048  # readable bytes required past the end of the cs buffer (mpc.h)
FLANK_PAD = 16  # readable bytes required past the end of the up/down buffers (mpc.h)


class MpcError(RuntimeError):
    pass


class DataError(Exception):
    """Input the reference rejects (exit status 1).  ``flags`` are MPC_DE_* bits."""

    def __init__(self, flags, read):
        names = [v for k, v in DE_NAMES.items() if flags & k]
        super().__init__(f"{'/'.join(names)} (first offending read index {read})")
        self.flags = flags
        self.read = read


class PlanInfo(ctypes.Structure):
    """mpc_plan_info (include/mpc.h): the geometry the planner chose."""
    _fields_ = [
        ("tally_mode", ctypes.c_int32), ("parse_window", ctypes.c_int32), ("parse_waves", ctypes.c_int32),
        ("parse_lds_bytes", ctypes.c_int32), ("parse_workgroups", ctypes.c_int32), ("overrides", ctypes.c_int32),
        ("max_reads_per_workgroup", ctypes.c_int64), ("reads_per_workgroup_cap", ctypes.c_int64),
        ("workspace_bytes", ctypes.c_int64), ("deferred_placement", ctypes.c_int32), ("reserved", ctypes.c_int32),
    ]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class _Input(ctypes.Structure):
    _fields_ = [
        ("ref", ctypes.c_void_p), ("ref_off", ctypes.c_void_p),
        ("cs", ctypes.c_void_p), ("cs_off", ctypes.c_void_p),
        ("tstart", ctypes.c_void_p),
        ("up", ctypes.c_void_p), ("up_off", ctypes.c_void_p),
        ("down", ctypes.c_void_p), ("down_off", ctypes.c_void_p),
        ("sample", ctypes.c_void_p),
        ("n_samples", ctypes.c_int32),
        ("h_ref_len", ctypes.POINTER(ctypes.c_int64)),
        ("h_read_begin", ctypes.POINTER(ctypes.c_int64)),
        ("n_reads", ctypes.c_int64),
        ("cs_bytes", ctypes.c_int64),
        ("cs_base", ctypes.c_int64),
        ("read_offset", ctypes.c_int64),
        ("n_reads_global", ctypes.c_int64),
        ("shard", ctypes.c_int32),
        ("n_shards", ctypes.c_int32),
        ("h_cs_off", ctypes.POINTER(ctypes.c_int64)),
        ("parse_cus", ctypes.c_int32),
        ("neg_reads", ctypes.c_int64),
        ("neg_cs_bytes", ctypes.c_int64),
    ]


_lib = None


def _hip_runtime_paths():
    """Distinct files of the HIP runtime (libamdhip64) mapped into this process."""
    paths = set()
    try:
        with open("/proc/self/maps") as f:
            for line in f:
                p = line.split()[-1] if line.strip() else ""
                if os.path.basename(p).startswith("libamdhip64.so"):
                    paths.add(os.path.realpath(p))
    except OSError:
        pass
    return paths


def _elf_dynamic(path):
    """(SONAME, [NEEDED...]) of an ELF64 little-endian shared library, from its
    .dynamic section (no tools, no loading; only the ELF header, the section
    headers and the .dynamic / string-table ranges are read); (None, []) if
    unreadable."""
    import struct
    try:
        with open(path, "rb") as f:
            def at(off, n):
                f.seek(off)
                b = f.read(n)
                if len(b) != n:
                    raise ValueError("short read")
                return b
            hdr = at(0, 64)
            if hdr[:4] != b"\x7fELF" or hdr[4] != 2 or hdr[5] != 1:
                return None, []
            shoff, = struct.unpack_from("<Q", hdr, 0x28)
            shentsize, shnum = struct.unpack_from("<HH", hdr, 0x3A)
            sh = at(shoff, shentsize * shnum)
            secs = [struct.unpack_from("<IIQQQQIIQQ", sh, k * shentsize) for k in range(shnum)]
            dyn = next((x for x in secs if x[1] == 6), None)  # SHT_DYNAMIC
            if dyn is None:
                return None, []
            strtab = secs[dyn[6]]  # sh_link: its string table
            strs = at(strtab[4], strtab[5])
            dynb = at(dyn[4], dyn[5])
            sname = lambda o: strs[o: strs.index(b"\0", o)].decode()
            soname, needed = None, []
            for k in range(len(dynb) // 16):
                tag, val = struct.unpack_from("<qQ", dynb, 16 * k)
                if tag == 0:
                    break
                if tag == 14:
                    soname = sname(val)
                elif tag == 1:
                    needed.append(sname(val))
            return soname, needed
    except (OSError, ValueError, struct.error, IndexError, StopIteration, UnicodeDecodeError):
        return None, []


def _torch_hip_runtime():
    """Path of PyTorch's own libamdhip64.so (torch/lib), without importing torch."""
    import importlib.util
    spec = importlib.util.find_spec("torch")
    if spec is None or not spec.origin:
        return None
    path = os.path.join(os.path.dirname(spec.origin), "lib", "libamdhip64.so")
    return path if os.path.exists(path) else None


def _preload_hip_runtime():
    """libmpc.so needs libamdhip64.so.N (NEEDED).  PyTorch-ROCm ships its own
    copy of that library with its own HSA runtime in torch/lib; two HIP/HSA
    runtimes in one process leave the second one with "no ROCm-capable
    device".  When PyTorch's copy has the SONAME libmpc.so needs, map it first
    (RTLD_GLOBAL, by path, without importing torch): the dynamic linker then
    binds libmpc.so's dependency to it by SONAME, and a later ``import torch``
    finds the same file already mapped -- one runtime in either import order.
    When the SONAMEs differ (a PyTorch built against another HIP major) the
    two cannot be shared: raise before anything is loaded or initialised
    (loading libmpc.so would map a second runtime).  Without PyTorch (a C-ABI
    user) the system ROCm copy is used."""
    path = _torch_hip_runtime()
    if path is None:
        return
    torch_so, _ = _elf_dynamic(path)
    need = next((x for x in _elf_dynamic(LIB_PATH)[1] if x.startswith("libamdhip64.so")), None)
    if torch_so is not None and need is not None and torch_so != need:
        raise MpcError("libmpc.so needs %s but PyTorch ships %s: two HIP runtimes cannot share this process; "
                       "rebuild libmpc.so against PyTorch's HIP" % (need, torch_so))
    ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise MpcError(f"{LIB_PATH} is missing: build it with __graft_entry__.build() (no CPU fallback)")
        _preload_hip_runtime()
        L = ctypes.CDLL(LIB_PATH)
        rt = _hip_runtime_paths()
        if len(rt) > 1:
            raise MpcError("two HIP runtimes are mapped into this process (%s): load libmpc.so through "
                           "engine.lib() before anything else loads a HIP runtime" % ", ".join(sorted(rt)))
        vp, i64, i32, dbl = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_double
        L.mpc_version.restype = i32
        L.mpc_last_error.restype = ctypes.c_char_p
        L.mpc_plan_create.argtypes = [ctypes.POINTER(_Input), i64, ctypes.POINTER(vp)]
        L.mpc_plan_destroy.argtypes = [vp]
        L.mpc_plan_workspace_bytes.argtypes = [vp, ctypes.POINTER(ctypes.c_size_t)]
        L.mpc_plan_bind.argtypes = [vp, vp, ctypes.c_size_t]
        L.mpc_plan_buffer.argtypes = [vp, i32, ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(i64)]
        L.mpc_plan_set_input.argtypes = [vp, ctypes.POINTER(_Input)]
        L.mpc_plan_get_info.argtypes = [vp, ctypes.POINTER(PlanInfo)]
        L.mpc_input_layout.argtypes = [ctypes.POINTER(ctypes.c_size_t), i32]
        L.mpc_input_layout.restype = ctypes.c_size_t
        for f in PHASES:
            getattr(L, "mpc_" + f).argtypes = [vp, vp]
        L.mpc_consensus.argtypes = [vp, dbl, dbl, vp]
        L.mpc_run.argtypes = [vp, dbl, dbl, vp]
        L.mpc_profile_kernel.argtypes = [vp, i32, vp]
        L.mpc_profile_kernel.restype = i32
        for f in ("mpc_plan_create", "mpc_plan_destroy", "mpc_plan_workspace_bytes", "mpc_plan_bind",
                  "mpc_plan_buffer", "mpc_plan_set_input", "mpc_plan_get_info", "mpc_consensus", "mpc_run") + tuple("mpc_" + x for x in PHASES):
            getattr(L, f).restype = i32
        if L.mpc_version() != ABI_VERSION:
            raise MpcError(f"{LIB_PATH}: ABI {L.mpc_version()} != {ABI_VERSION} (rebuild)")
        _lib = L
    return _lib


def set_library(path):
    """Experiments only (scripts/): load a variant build of libmpc.so instead of
    the in-tree one.  Must be called before the first lib() call."""
    global LIB_PATH
    if _lib is not None:
        raise MpcError("libmpc.so is already loaded")
    LIB_PATH = path


def geometry(ref_lens, reads_per_sample, cs_bytes, n_reads_global=None, read_offset=0, shard=0, n_shards=1,
             parse_cus=0, neg_reads=0):
    """Host-only planning (no device): the mpc_plan_info a Plan over inputs of
    this shape would use (``parse_cus`` as for Batch; ``neg_reads``: reads with
    a negative tstart).  Needs no GPU."""
    ref_len = np.ascontiguousarray(ref_lens, dtype=np.int64)
    counts = np.asarray(reads_per_sample, dtype=np.int64)
    rb = np.ascontiguousarray(np.concatenate([[0], np.cumsum(counts)]), dtype=np.int64)
    n = int(rb[-1])
    inp = _Input(n_samples=len(ref_len), h_ref_len=ref_len.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                 h_read_begin=rb.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), n_reads=n, cs_bytes=int(cs_bytes),
                 cs_base=0, read_offset=read_offset, n_reads_global=n_reads_global or n, shard=shard,
                 n_shards=n_shards, parse_cus=int(parse_cus), neg_reads=int(neg_reads))
    L = lib()
    h = ctypes.c_void_p()
    _check(L.mpc_plan_create(ctypes.byref(inp), int((4 * ref_len + 8).sum() + 1024), ctypes.byref(h)))
    try:
        info = PlanInfo()
        _check(L.mpc_plan_get_info(h, ctypes.byref(info)))
        return info.as_dict()
    finally:
        L.mpc_plan_destroy(h)


PARSE_CHUNKS = 48  # include/mpc.h MPC_PARSE_CHUNKS


def parse_split(ref_lens, reads_per_sample, cs_off):
    """Host-only (no device): the parse work split a Plan over these reads
    would launch -- (work int32[n_wg, 4] = sample, first read, end read,
    chunks; chunks int32[n_wg, PARSE_CHUNKS + 1] read boundaries)."""
    ref_len = np.ascontiguousarray(ref_lens, dtype=np.int64)
    counts = np.asarray(reads_per_sample, dtype=np.int64)
    rb = np.ascontiguousarray(np.concatenate([[0], np.cumsum(counts)]), dtype=np.int64)
    off = np.ascontiguousarray(cs_off, dtype=np.int64)
    n = int(rb[-1])
    assert off.shape == (n + 1,)
    p64 = ctypes.POINTER(ctypes.c_int64)
    inp = _Input(n_samples=len(ref_len), h_ref_len=ref_len.ctypes.data_as(p64), h_read_begin=rb.ctypes.data_as(p64),
                 n_reads=n, cs_bytes=int(off[-1]), cs_base=0, read_offset=0, n_reads_global=n, shard=0, n_shards=1,
                 h_cs_off=off.ctypes.data_as(p64))
    L = lib()
    L.mpc_plan_parse_tables.argtypes = [ctypes.c_void_p] * 3
    h = ctypes.c_void_p()
    _check(L.mpc_plan_create(ctypes.byref(inp), int((4 * ref_len + 8).sum() + 1024), ctypes.byref(h)))
    try:
        n_wg = L.mpc_plan_parse_tables(h, None, None)
        if n_wg < 0:
            _check(n_wg)
        work = np.zeros((n_wg, 4), np.int32)
        chunks = np.zeros((n_wg, PARSE_CHUNKS + 1), np.int32)
        _check(L.mpc_plan_parse_tables(h, work.ctypes.data, chunks.ctypes.data) - n_wg)
        return work, chunks
    finally:
        L.mpc_plan_destroy(h)


def _check(rc):
    if rc != 0:
        raise MpcError(f"libmpc error {rc}: {lib().mpc_last_error().decode(errors='replace')}")


def _torch():
    import torch
    return torch


class Batch:
    """Device-resident inputs of one launch: one or more samples (strands /
    plasmids) concatenated, reads grouped by sample."""

    def __init__(self, samples, device=0, read_offset=0, n_reads_global=None, shard=0, n_shards=1,
                 balance_bytes=True, parse_cus=0):
        """``balance_bytes``: hand the planner the host cs offsets so the parse
        work is split by cs bytes (mpc.h h_cs_off); False splits by read count.
        ``parse_cus``: CUs the parse grid is sized for (0: all; mpc.h parse_cus),
        fewer when other batches are in flight beside this one."""
        torch = _torch()
        if not torch.cuda.is_available():
            raise MpcError("no HIP device visible (the pileup path has no CPU fallback)")
        self.device = torch.device("cuda", device)
        S = len(samples)
        self.n_samples = S
        self.ref_len = np.array([len(s["ref"]) for s in samples], dtype=np.int64)
        counts = np.array([len(s["tstart"]) for s in samples], dtype=np.int64)
        self.read_begin = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
        self.n_reads = int(self.read_begin[-1])
        self.read_offset = int(read_offset)
        self.n_reads_global = int(n_reads_global if n_reads_global is not None else self.n_reads)
        self.shard, self.n_shards = int(shard), int(n_shards)
        self.parse_cus = int(parse_cus)

        def cat_bytes(key, offkey):
            if S == 1:  # one sample: its buffer as is (no copy of a GB of cs)
                b = np.asarray(samples[0][key], dtype=np.uint8)
                o = np.asarray(samples[0][offkey], dtype=np.int64)
                if len(o) and o[0] == 0:
                    return b[:o[-1]], o
            bufs, offs, base = [], [], 0
            for s in samples:
                b = np.asarray(s[key], dtype=np.uint8)
                o = np.asarray(s[offkey], dtype=np.int64)
                bufs.append(b[o[0]:o[-1]] if len(o) else b[:0])
                offs.append((o[:-1] - o[0] + base) if len(o) else o)
                base += (o[-1] - o[0]) if len(o) else 0
            data = np.concatenate(bufs) if bufs else np.zeros(0, np.uint8)
            off = np.concatenate(offs + [np.array([base], dtype=np.int64)])
            return data, off

        cs, cs_off = cat_bytes("cs", "cs_off")
        up, up_off = cat_bytes("up", "up_off")
        dn, dn_off = cat_bytes("down", "down_off")
        refs = [np.asarray(s["ref"], dtype=np.uint8) for s in samples]
        ref = np.concatenate(refs) if refs else np.zeros(0, np.uint8)
        ref_off = np.concatenate([[0], np.cumsum([len(r) for r in refs])]).astype(np.int64)
        tstart = np.concatenate([np.asarray(s["tstart"], dtype=np.int64) for s in samples])
        if len(tstart) and (tstart.min() < -(2 ** 31) or tstart.max() >= 2 ** 31):
            raise MpcError("target start out of int32 range")
        sample = np.repeat(np.arange(S, dtype=np.int32), counts)
        self.cs_bytes = int(cs_off[-1])
        # reads with a negative target start (Python's negative wrap, mpc.h): they
        # size the plan's list of strings written into wrapped odd positions
        neg = tstart < 0
        self.neg_reads = int(neg.sum())
        self.neg_cs_bytes = int((cs_off[1:] - cs_off[:-1])[neg].sum()) if self.neg_reads else 0
        self.aligned_bases = int(sum(int(np.asarray(s.get("aligned", [0])).sum()) for s in samples))

        def dev(a, pad=0):
            a = np.ascontiguousarray(a)
            t = torch.empty(max(a.nbytes + pad, 16), dtype=torch.uint8, device=self.device)
            if a.nbytes:
                # (read-only views of the ingest's buffers are only read here: the
                # host tensor is the source of one H2D copy, never written)
                with warnings.catch_warnings():
                    warnings.filterwarnings("ignore", message="The given NumPy array is not writable")
                    h = torch.from_numpy(a.view(np.uint8).reshape(-1))
                t[: a.nbytes].copy_(h)
            if pad:
                t[a.nbytes:].zero_()
            return t

        self.t = dict(
            ref=dev(ref), ref_off=dev(ref_off), cs=dev(cs, CS_PAD), cs_off=dev(cs_off),
            tstart=dev(tstart.astype(np.int32)), up=dev(up, FLANK_PAD), up_off=dev(up_off),
            down=dev(dn, FLANK_PAD), down_off=dev(dn_off), sample=dev(sample),
        )
        self.h_cs_off = cs_off
        self.balance_bytes = bool(balance_bytes)
        self.max_flank = int(max((np.diff(up_off).max() if len(up_off) > 1 else 0),
                                 (np.diff(dn_off).max() if len(dn_off) > 1 else 0)))

    def c_input(self):
        t = self.t
        self._keep = (np.ascontiguousarray(self.ref_len), np.ascontiguousarray(self.read_begin),
                      np.ascontiguousarray(self.h_cs_off, dtype=np.int64))
        return _Input(
            ref=t["ref"].data_ptr(), ref_off=t["ref_off"].data_ptr(), cs=t["cs"].data_ptr(),
            cs_off=t["cs_off"].data_ptr(), tstart=t["tstart"].data_ptr(), up=t["up"].data_ptr(),
            up_off=t["up_off"].data_ptr(), down=t["down"].data_ptr(), down_off=t["down_off"].data_ptr(),
            sample=t["sample"].data_ptr(), n_samples=self.n_samples,
            h_ref_len=self._keep[0].ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
            h_read_begin=self._keep[1].ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
            n_reads=self.n_reads, cs_bytes=self.cs_bytes, cs_base=0,
            read_offset=self.read_offset, n_reads_global=self.n_reads_global,
            shard=self.shard, n_shards=self.n_shards,
            h_cs_off=(self._keep[2].ctypes.data_as(ctypes.POINTER(ctypes.c_int64)) if self.balance_bytes
                      else ctypes.POINTER(ctypes.c_int64)()),
            parse_cus=int(self.parse_cus), neg_reads=self.neg_reads, neg_cs_bytes=self.neg_cs_bytes,
        )

    def row_estimate(self):
        n = self.ref_len
        return int((4 * n + 8).sum() + 4 * self.max_flank * self.n_samples + 1024)


class Plan:
    """A bound plan: one workspace for one Batch shape."""

    def __init__(self, batch, row_cap=None):
        torch = _torch()
        self.batch = batch
        self.row_cap = int(row_cap or batch.row_estimate())
        L = lib()
        self._inp = batch.c_input()
        h = ctypes.c_void_p()
        _check(L.mpc_plan_create(ctypes.byref(self._inp), self.row_cap, ctypes.byref(h)))
        self.h = h
        nb = ctypes.c_size_t()
        _check(L.mpc_plan_workspace_bytes(h, ctypes.byref(nb)))
        self.ws_bytes = nb.value
        self.ws_raw = torch.empty(self.ws_bytes + 256, dtype=torch.uint8, device=batch.device)
        pad = (-self.ws_raw.data_ptr()) % 256
        self.ws = self.ws_raw[pad: pad + self.ws_bytes]
        self._views = {}
        _check(L.mpc_plan_bind(h, ctypes.c_void_p(self.ws.data_ptr()), self.ws_bytes))

    def __del__(self):
        h = getattr(self, "h", None)
        if h is not None and _lib is not None:
            _lib.mpc_plan_destroy(h)
            self.h = None

    def info(self):
        info = PlanInfo()
        _check(lib().mpc_plan_get_info(self.h, ctypes.byref(info)))
        return info.as_dict()

    def buffer(self, which, dtype):
        """View of one workspace buffer (memoized: the binding never moves)."""
        key = ("b", which, dtype)
        v = self._views.get(key)
        if v is None:
            v = self._views[key] = self._buffer(which, dtype)
        return v

    def _buffer(self, which, dtype):
        torch = _torch()
        off, cnt = ctypes.c_size_t(), ctypes.c_int64()
        _check(lib().mpc_plan_buffer(self.h, which, ctypes.byref(off), ctypes.byref(cnt)))
        item = torch.empty(0, dtype=dtype).element_size()
        return self.ws[off.value: off.value + cnt.value * item].view(dtype)

    def span(self, first, last, dtype):
        """The workspace bytes from buffer ``first`` through buffer ``last``
        (include/mpc.h: buffers exchanged together are laid out in order)."""
        key = ("s", first, last, dtype)
        v = self._views.get(key)
        if v is None:
            v = self._views[key] = self._span(first, last, dtype)
        return v

    def _span(self, first, last, dtype):
        torch = _torch()
        o0, c0, o1, c1 = ctypes.c_size_t(), ctypes.c_int64(), ctypes.c_size_t(), ctypes.c_int64()
        _check(lib().mpc_plan_buffer(self.h, first, ctypes.byref(o0), ctypes.byref(c0)))
        _check(lib().mpc_plan_buffer(self.h, last, ctypes.byref(o1), ctypes.byref(c1)))
        item = torch.empty(0, dtype=dtype).element_size()
        end = o1.value + c1.value * item
        if o1.value < o0.value or (end - o0.value) % item:
            raise MpcError("buffers %d..%d are not an ordered span" % (first, last))
        return self.ws[o0.value: end].view(dtype)

    def stream_ptr(self, stream=None):
        torch = _torch()
        s = stream if stream is not None else torch.cuda.current_stream(self.batch.device)
        return ctypes.c_void_p(s.cuda_stream)

    def run(self, mdf, gtf, stream=None):
        _check(lib().mpc_run(self.h, float(mdf), float(gtf), self.stream_ptr(stream)))

    def profile_kernel(self, which, stream=None):
        _check(lib().mpc_profile_kernel(self.h, int(which), self.stream_ptr(stream)))

    def phase(self, name, stream=None, *args):
        fn = getattr(lib(), "mpc_" + name)
        if name == "consensus":
            _check(fn(self.h, float(args[0]), float(args[1]), self.stream_ptr(stream)))
        else:
            _check(fn(self.h, self.stream_ptr(stream)))

    def status(self):
        torch = _torch()
        return self.buffer(BUF_STATUS, torch.int32).cpu().numpy().view(np.uint32)

    def fetch(self):
        """Copy the calls of every sample to the host.  Raises DataError when
        the reference would have failed on this input."""
        torch = _torch()
        st = self.status()
        flags = int(st[MPC_ST_FLAGS])
        if flags:
            raise DataError(flags, int(st[MPC_ST_FIRST_READ]))
        nc = self.buffer(BUF_NCALLS, torch.int32).cpu().numpy()
        total = int(nc[-1])
        calls = self.buffer(BUF_CALLS, torch.int32)[: total * 4].cpu().numpy().view(np.uint32).reshape(-1, 4)
        md = self.buffer(BUF_MAXDEPTH, torch.int32).cpu().numpy().view(np.uint32)
        out = []
        for s in range(self.batch.n_samples):
            c = calls[nc[s]: nc[s + 1]]
            out.append(dict(
                raw=np.ascontiguousarray(c),  # the device rows (include/mpc.h MPC_BUF_CALLS), for the native writers
                base=(c[:, 0] & 0xFF).astype(np.uint8), chrom1=((c[:, 0] >> 8) & 0xFF).astype(np.uint8),
                chrom2=((c[:, 0] >> 16) & 0xFF).astype(np.uint8), count=c[:, 1].astype(np.int64),
                count2=c[:, 2].astype(np.int64), total=c[:, 3].astype(np.int64), max_depth=int(md[s]),
            ))
        return out


def pileup(samples, mdf, gtf, device=0, row_cap=None):
    """One-shot helper: samples (packed dicts) -> per-sample call dicts.
    Re-plans once if the row capacity estimate was too small."""
    torch = _torch()
    batch = Batch(samples, device=device)
    plan = Plan(batch, row_cap)
    plan.run(mdf, gtf)
    st = plan.status()
    flags = int(st[MPC_ST_FLAGS])
    if flags & DE_CAPACITY and not (flags & ~DE_CAPACITY):
        need = int(st[MPC_ST_ROWS_NEEDED])
        plan = Plan(batch, need + 16)
        plan.run(mdf, gtf)
    res = plan.fetch()
    torch.cuda.synchronize(batch.device)
    return res


class Runner:
    """Repeated pileups over one device-resident Batch (bench / serving loop).
    The first step sizes the row buffers exactly (re-plans once if needed)."""

    def __init__(self, samples, device=0, row_cap=None, parse_cus=0):
        self.batch = Batch(samples, device=device, parse_cus=parse_cus)
        self.plan = Plan(self.batch, row_cap)
        self._sized = False

    def step(self, mdf, gtf, stream=None):
        self.plan.run(mdf, gtf, stream)
        if not self._sized:
            st = self.plan.status()
            flags = int(st[MPC_ST_FLAGS])
            if flags & DE_CAPACITY and not (flags & ~DE_CAPACITY):
                self.plan = Plan(self.batch, int(st[MPC_ST_ROWS_NEEDED]) + 16)
                self.plan.run(mdf, gtf, stream)
            self._sized = True

    def check(self):
        st = self.plan.status()
        if int(st[MPC_ST_FLAGS]):
            raise DataError(int(st[MPC_ST_FLAGS]), int(st[MPC_ST_FIRST_READ]))

    def fetch(self):
        return self.plan.fetch()
