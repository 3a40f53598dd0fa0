"""Seeded synthetic cs-tagged alignments (ctypes wrapper over csrc/synth.cpp).

Profiles follow SURVEY.md §8(d): uniform ACGT plasmid, i.i.d. per-base
sub/ins/del, indel lengths 1-3, flanks 0-40 nt, 2 % partial alignments,
50 % minus strand; sample 1 is the same reads aligned to revcomp(ref)
(the antisense assembly of Snakefile:348-378).
"""
import ctypes
import os

import numpy as np

from . import _build

(REF, CS, CS_OFF, TSTART, UP, UP_OFF, DOWN, DOWN_OFF, ALIGNED, STRAND, TEND) = range(11)


class _Params(ctypes.Structure):
    _fields_ = [
        ("n", ctypes.c_int64), ("n_reads", ctypes.c_int64),
        ("p_sub", ctypes.c_double), ("p_ins", ctypes.c_double), ("p_del", ctypes.c_double),
        ("ins_min", ctypes.c_int32), ("ins_max", ctypes.c_int32),
        ("del_min", ctypes.c_int32), ("del_max", ctypes.c_int32),
        ("flank_min", ctypes.c_int32), ("flank_max", ctypes.c_int32),
        ("frac_partial", ctypes.c_double), ("frac_minus", ctypes.c_double),
        ("seed", ctypes.c_uint64), ("antisense", ctypes.c_int32), ("n_threads", ctypes.c_int32),
        ("read_begin", ctypes.c_int64), ("read_end", ctypes.c_int64),
    ]


PROFILES = {
    # SURVEY.md §8(d) default profile
    "default": dict(p_sub=0.01, p_ins=0.005, p_del=0.005),
    # §8(d) indel-heavy (R10.3-like, BASELINE.json configs[3])
    "indel": dict(p_sub=0.01, p_ins=0.05, p_del=0.05),
    # the 2/2/2 % profile of the survey's C1 probe
    "c1probe": dict(p_sub=0.02, p_ins=0.02, p_del=0.02),
}

_lib = None


def lib():
    global _lib
    if _lib is None:
        path = _build.ensure_synth()
        L = ctypes.CDLL(path)
        L.mpc_synth_new.restype = ctypes.c_void_p
        L.mpc_synth_new.argtypes = [ctypes.POINTER(_Params)]
        L.mpc_synth_free.argtypes = [ctypes.c_void_p]
        L.mpc_synth_size.restype = ctypes.c_int64
        L.mpc_synth_size.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
        L.mpc_synth_copy.restype = ctypes.c_int
        L.mpc_synth_copy.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
        L.mpc_synth_write_files.restype = ctypes.c_int
        L.mpc_synth_write_files.argtypes = [ctypes.c_void_p] + [ctypes.c_char_p] * 5
        _lib = L
    return _lib


class Synth:
    """One generated data set (1 or 2 samples).  ``sample(s)`` returns the packed
    inputs exactly as the host ingest produces them from the written files."""

    def __init__(self, n, n_reads, profile="default", seed=1, antisense=True, frac_partial=0.02,
                 frac_minus=0.5, ins_len=(1, 3), del_len=(1, 3), flank=(0, 40), n_threads=0, reads=None, **over):
        """``reads=(a, b)``: only reads [a, b) of the ``n_reads``-read set, each
        identical to the same read of the full set (multi-GPU shards)."""
        pr = dict(PROFILES[profile])
        pr.update(over)
        p = _Params(n=n, n_reads=n_reads, p_sub=pr["p_sub"], p_ins=pr["p_ins"], p_del=pr["p_del"],
                    ins_min=ins_len[0], ins_max=ins_len[1], del_min=del_len[0], del_max=del_len[1],
                    flank_min=flank[0], flank_max=flank[1], frac_partial=frac_partial,
                    frac_minus=frac_minus, seed=seed, antisense=1 if antisense else 0,
                    n_threads=n_threads, read_begin=reads[0] if reads else 0, read_end=reads[1] if reads else 0)
        self.params = p
        self.n_samples = 2 if antisense else 1
        self._h = lib().mpc_synth_new(ctypes.byref(p))

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            lib().mpc_synth_free(h)
            self._h = None

    def _get(self, what, s, dtype):
        L = lib()
        nb = L.mpc_synth_size(self._h, what, s)
        a = np.empty(nb // np.dtype(dtype).itemsize, dtype=dtype)
        if nb:
            L.mpc_synth_copy(self._h, what, s, a.ctypes.data)
        return a

    def sample(self, s=0):
        return dict(
            ref=self._get(REF, s, np.uint8),
            cs=self._get(CS, s, np.uint8), cs_off=self._get(CS_OFF, s, np.int64),
            tstart=self._get(TSTART, s, np.int64),
            up=self._get(UP, s, np.uint8), up_off=self._get(UP_OFF, s, np.int64),
            down=self._get(DOWN, s, np.uint8), down_off=self._get(DOWN_OFF, s, np.int64),
            aligned=self._get(ALIGNED, s, np.int64), tend=self._get(TEND, s, np.int64),
        )

    def write_files(self, ref_fa=None, reads_fa=None, paf0=None, ref_as_fa=None, paf1=None):
        enc = lambda x: x.encode() if x else None
        rc = lib().mpc_synth_write_files(self._h, enc(ref_fa), enc(reads_fa), enc(paf0), enc(ref_as_fa), enc(paf1))
        if rc != 0:
            raise OSError("synth write failed")
