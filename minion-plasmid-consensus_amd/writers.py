"""Step 7 writers of the reference (:446-463), fed by the device call arrays.

consensus  ">consensus\\n" + called bases + "\\n"
chromat    "pos\\tbase\\tcount" header, two lines per call (top, second) using the
           pre-GTF bases; pos is the 1-based index in the consensus
accuracies "pos\\taccuracy" header, str(100 * (count / total)) per call

The CLI writes through the native writer (csrc/writers.cpp, libmpc_ingest.so:
all cores, Python float repr restated); the text functions below are the same
formats in Python (tests compare the two).
"""
import os

import numpy as np


def consensus_text(calls):
    return ">consensus\n" + bytes(calls["base"]).decode("ascii") + "\n"


def chromat_text(calls):
    c1 = bytes(calls["chrom1"]).decode("ascii")
    c2 = bytes(calls["chrom2"]).decode("ascii")
    cnt = calls["count"].tolist()
    cnt2 = calls["count2"].tolist()
    out = ["pos\tbase\tcount\n"]
    for i in range(len(cnt)):
        out.append("%d\t%s\t%d\n%d\t%s\t%d\n" % (i + 1, c1[i], cnt[i], i + 1, c2[i], cnt2[i]))
    return "".join(out)


def accuracies_text(calls):
    # 100 * (count / total): the division of two ints < 2^53 is the correctly
    # rounded IEEE quotient in both Python and numpy, then one f64 multiply;
    # str() of a Python float is the shortest round-trip repr (:431, :463).
    cnt = np.asarray(calls["count"], dtype=np.float64)
    tot = np.asarray(calls["total"], dtype=np.float64)
    acc = (100.0 * (cnt / tot)).tolist() if len(cnt) else []
    out = ["pos\taccuracy\n"]
    out.extend("{}\t{}\n".format(i + 1, a) for i, a in enumerate(acc))
    return "".join(out)


class WriteError(OSError):
    pass


def write_outputs(calls, consensus_path, chromat_path, accuracies_path, n_threads=0):
    """The three output files of one sample, from its device calls (``calls["raw"]``,
    engine.Plan.fetch) through the native writer."""
    import ctypes
    from . import ingest
    L = ingest._native()
    if L is None:  # no host compiler to build the native writers: same formats in Python
        write_outputs_python(calls, consensus_path, chromat_path, accuracies_path)
        return
    raw = np.ascontiguousarray(calls["raw"], dtype=np.uint32).reshape(-1, 4)
    msg = ctypes.create_string_buffer(256)
    buf = raw if raw.size else np.zeros((1, 4), np.uint32)
    rc = L.mpc_write_calls(buf.ctypes.data, len(raw), os.fsencode(consensus_path), os.fsencode(chromat_path),
                           os.fsencode(accuracies_path), int(n_threads), msg, 256)
    if rc != 0:
        raise WriteError(msg.value.decode(errors="replace"))


def write_outputs_python(calls, consensus_path, chromat_path, accuracies_path):
    """The same files through the Python text functions (tests, call dicts without ``raw``)."""
    with open(consensus_path, "w") as f:
        f.write(consensus_text(calls))
    with open(chromat_path, "w") as f:
        f.write(chromat_text(calls))
    with open(accuracies_path, "w") as f:
        f.write(accuracies_text(calls))


def py_float_repr(x):
    """repr(x) as the native writer prints it (tests)."""
    import ctypes
    from . import ingest
    out = ctypes.create_string_buffer(40)
    n = ingest._native().mpc_py_float_repr(float(x), out, 40)
    return out.value[:n].decode()


# Snakefile:77 (the rule's own table; no lower case, no 'X')
_COMPLEMENT = {"A": "T", "T": "A", "G": "C", "C": "G", "N": "N"}


class RevcompError(ValueError):
    pass


def revcomp_text(lines):
    """Rule `revcomp_antisense_consensus` (Snakefile:425-450) on a list of lines
    (each with its newline, as file iteration yields them): every '>' line is
    copied; then the reverse complement of the LAST line only (rstripped,
    upper-cased) is appended without a newline (:445, the rule uses the loop
    variable, not the accumulated sequence).  Returns (text, error): on a base
    outside A/C/G/T/N or an empty file the rule raises after the header lines
    were written, so the partial text is returned with the error."""
    head = "".join(ln for ln in lines if ln.startswith(">"))
    if not lines:
        return head, RevcompError("NameError: name 'line' is not defined")  # empty input: loop never ran
    out = []
    for x in lines[-1].rstrip()[::-1]:
        c = _COMPLEMENT.get(x.upper())
        if c is None:
            return head, RevcompError("KeyError: {!r}".format(x.upper()))
        out.append(c)
    return head + "".join(out), None


def revcomp_consensus(src_path, dst_path):
    """File form of revcomp_text; raises RevcompError like the rule (exit 1)
    after writing the header lines."""
    with open(src_path, "r") as f:
        lines = f.readlines()
    text, err = revcomp_text(lines)
    with open(dst_path, "w") as f:
        f.write(text)
    if err is not None:
        raise err
