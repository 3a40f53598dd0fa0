"""Drop-in for src/pseudopair_reads.py (rule pseudopair_reads, Snakefile:211-228).

Same flags, same output file, same exit status.  Reads the PAF of the initial
alignment and pairs forward-strand with reverse-strand reads for duplex
basecalling:

  * a read name seen for the first time goes to the forward table (strand
    field exactly "+") or the reverse table (anything else) with its aligned
    length qend - qstart (:96-115)
  * seeing the name again deletes it from its table; a third sighting adds it
    again, at the end of the table order (dict delete / re-insert, :103-110)
  * reads with aligned length < --min_align_length are dropped (:119-133)
  * the output pairs the i-th surviving forward read with the i-th surviving
    reverse read, "fwd rev" per line, until the shorter table ends (:137-140)

The PAF is parsed by the native host library (csrc/pseudopair.cpp, memory-
mapped, all cores for the line parsing); inputs with integers in a form only
Python's int() accepts, non-ASCII bytes or carriage returns are declined by
it and handled by :func:`pseudopair_python`, which restates the script.
Errors the script raises (a line with fewer than 5 fields, int() failures, a
missing --min_align_length with reads left) exit 1 with no output file, as
the script fails before it opens the output.
"""
import argparse
import ctypes
import os
import sys
import time

TITLE = "PseudoPair Reads"


class PairError(Exception):
    """An input the reference rejects (exit status 1)."""


def statprint(msg, msg_type="STATUS"):
    print("\033[1;37;40m{}\033[0m \033[1;34;40m[{}]\033[0m: {}".format(msg_type, time.strftime("%Y/%m/%d %T"), msg),
          flush=True)


def pseudopair_python(paf_path, min_align_length):
    """Returns (pairs, n_fwd, n_rev, n_fwd_kept, n_rev_kept) like the script (:92-140)."""
    fwd, rev = {}, {}
    with open(paf_path, "r") as fh:
        for line in fh:
            f = line.split("\t")
            try:
                name = f[0]
                int(f[1])  # read length: parsed (and so validated) but unused (:97)
                length = int(f[3]) - int(f[2])
                strand = f[4]
            except (IndexError, ValueError) as e:
                raise PairError("{}: {}".format(type(e).__name__, e))
            if name in fwd:
                del fwd[name]
            elif name in rev:
                del rev[name]
            elif strand == "+":
                fwd[name] = length
            else:
                rev[name] = length
    n_fwd, n_rev = len(fwd), len(rev)
    if (fwd or rev) and min_align_length is None:
        raise PairError("TypeError: '<' not supported between instances of 'int' and 'NoneType'")
    fwd = [k for k, v in fwd.items() if not v < min_align_length]
    rev = [k for k, v in rev.items() if not v < min_align_length]
    return list(zip(fwd, rev)), n_fwd, n_rev, len(fwd), len(rev)


class _Stats(ctypes.Structure):
    _fields_ = [("n_fwd", ctypes.c_int64), ("n_rev", ctypes.c_int64), ("n_fwd_kept", ctypes.c_int64),
                ("n_rev_kept", ctypes.c_int64), ("n_pairs", ctypes.c_int64), ("status", ctypes.c_int32),
                ("message", ctypes.c_char * 256)]


def _lib():
    from . import ingest
    L = ingest._native()
    if L is None:
        return None
    if not hasattr(L, "_pp_ready"):
        L.mpc_pseudopair.restype = ctypes.c_int
        L.mpc_pseudopair.argtypes = [ctypes.c_char_p, ctypes.c_int64, ctypes.c_int, ctypes.c_char_p, ctypes.c_int,
                                     ctypes.POINTER(_Stats)]
        L._pp_ready = True
    return L


def pseudopair_native(paf_path, min_align_length, out_path, n_threads=0):
    """The whole tool through libmpc_ingest.so: writes out_path and returns the
    stats, None when the native parser declines the input, or raises PairError."""
    L = _lib()
    if L is None:
        return None
    st = _Stats()
    L.mpc_pseudopair(os.fsencode(paf_path), int(min_align_length or 0), 0 if min_align_length is None else 1,
                     os.fsencode(out_path), int(n_threads), ctypes.byref(st))
    if st.status == 2:
        return None
    if st.status != 0:
        raise PairError(st.message.decode(errors="replace"))
    return st


def build_parser():
    p = argparse.ArgumentParser(description=TITLE)
    p.add_argument("--paf", help="Input paf file", type=str)
    p.add_argument("--min_align_length", help="Minimum alignment length to accept", type=int)
    p.add_argument("--pseudopairs", help="Output read pairs file", type=str)
    p.add_argument("-d", "--debug", action="store_true", dest="DEBUG", help="Flag for setting debug/test state.")
    p.add_argument("-v", "--verbose", action="store_true", dest="VERB", help="Flag for setting verbose output.")
    return p


def main(argv=None):
    args = build_parser().parse_args(argv)
    print("=======================================================")
    print("Python version: {}".format(sys.version))
    print("Python environment: {}".format(sys.prefix))
    print("Server: {}".format(os.uname()[1]))
    print("Current directory: {}".format(os.getcwd()))
    print("Command: {}".format(" ".join(sys.argv)))
    print("Time: {}".format(time.strftime("%Y/%m/%d %T")))
    print("=======================================================\n")
    statprint("Parsing PAF file...")
    try:
        st = pseudopair_native(args.paf, args.min_align_length, args.pseudopairs)
        if st is not None:
            counts = (st.n_fwd, st.n_rev, st.n_fwd_kept, st.n_rev_kept)
        else:
            pairs, *counts = pseudopair_python(args.paf, args.min_align_length)
    except (PairError, OSError, UnicodeDecodeError) as e:
        print("Error: {}".format(e), file=sys.stderr)
        return 1
    statprint("There are {} forward reads and {} reverse reads.".format(counts[0], counts[1]))
    statprint("Removing reads with short alignments...")
    statprint("There are {} forward reads and {} reverse reads.".format(counts[2], counts[3]))
    statprint("Pseudopairing...")
    if st is None:
        with open(args.pseudopairs, "w") as out:
            out.write("".join("{} {}\n".format(fr, rr) for fr, rr in pairs))
    statprint("Done.")
    return 0


if __name__ == "__main__":
    sys.exit(main())
