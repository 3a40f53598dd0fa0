"""Seeded batches with negative target starts (minimap2 never writes one; the
reference indexes obsarr / refarr with Python's negative wrap,
mapped_paf_read_parser.py:222, :300-303, :57-61, :67-71, :79-97, :323).

A fraction of the reads start at tstart in [-n, -1] and take ':' / '*' / '+' /
'-' operations through the negative coordinates; some stay below 0 to their
end (downstream flank into the wrapped odd position n + i_end), the others
cross into the reference.  Starts and negative ends are drawn from a few values
so that wrapped odd positions collect several upstream flanks, '+' strings
and downstream flanks from reads in different orders, interleaved with the
one-base writes of the reads covering the same reference base.  Every batch
is valid input (the oracle raises nothing)."""
import numpy as np

ACGT = np.frombuffer(b"ACGT", dtype=np.uint8)


def _bases(rng, k, lower=False):
    s = bytes(rng.choice(ACGT, k))
    return s.lower() if lower else s


def _cs(rng, n, ts, stay_negative, neg_end):
    """cs of one read from coordinate ts; returns (cs bytes, end coordinate)."""
    out, i = [b"Z:"], ts
    if stay_negative:
        stop = neg_end
    else:
        stop = int(rng.integers(max(i + 1, 1), n + 1))
    while i < stop:
        r = rng.random()
        room = stop - i
        if r < 0.45:
            k = int(rng.integers(1, min(room, 25) + 1))
            out.append(b":%d" % k)
            i += k
        elif r < 0.6:
            out.append(b"*" + _bases(rng, 1, True) + _bases(rng, 1, rng.random() < 0.5))
            i += 1
        elif r < 0.8:
            out.append(b"+" + _bases(rng, int(rng.integers(1, 5)), rng.random() < 0.5))
        else:
            k = int(rng.integers(1, min(room, 3) + 1))
            out.append(b"-" + _bases(rng, k, True))
            i += k
    if rng.random() < 0.3:  # an insertion right at the end coordinate
        out.append(b"+" + _bases(rng, int(rng.integers(1, 4)), True))
    return b"".join(out), i


def neg_sample(seed, n=240, n_reads=2500, frac_neg=0.05, flank_max=6):
    """One sample dict (synth layout: ref, cs, cs_off, tstart, up, up_off,
    down, down_off, aligned)."""
    rng = np.random.default_rng(seed)
    ref = bytes(rng.choice(ACGT, n))
    starts = [-int(x) for x in rng.choice(np.arange(1, n + 1), 6, replace=False)]
    ends = [-int(x) for x in rng.choice(np.arange(1, n // 2), 4, replace=False)]
    cs, ts, ups, dns = [], [], [], []
    for _ in range(n_reads):
        if rng.random() < frac_neg:
            t = int(rng.choice(starts))
            e = [x for x in ends if x > t]
            stay = bool(e) and rng.random() < 0.5
            c, end = _cs(rng, n, t, stay, int(rng.choice(e)) if stay else 0)
        else:
            t = int(rng.integers(0, n - 1))
            c, end = _cs(rng, n, t, False, 0)
        cs.append(c)
        ts.append(t)
        ups.append(_bases(rng, int(rng.integers(0, flank_max + 1))))
        dns.append(_bases(rng, int(rng.integers(0, flank_max + 1))))
    off = lambda xs: np.concatenate([[0], np.cumsum([len(x) for x in xs])]).astype(np.int64)
    arr = lambda xs: np.frombuffer(b"".join(xs), dtype=np.uint8).copy()
    return dict(ref=np.frombuffer(ref, dtype=np.uint8).copy(), cs=arr(cs), cs_off=off(cs),
                tstart=np.asarray(ts, dtype=np.int64), up=arr(ups), up_off=off(ups), down=arr(dns),
                down_off=off(dns), aligned=np.zeros(n_reads, np.int64))


def wrapped_strings(smp):
    """(upstream, '+', downstream) strings the negative wrap writes into odd
    positions -- a host restatement of the rule, for the tests' coverage checks."""
    n = len(smp["ref"])
    up = down = ins = 0
    cs = bytes(smp["cs"])
    for r, t in enumerate(smp["tstart"]):
        t = int(t)
        ul = smp["up_off"][r + 1] - smp["up_off"][r]
        dl = smp["down_off"][r + 1] - smp["down_off"][r]
        up += int(ul > 0 and -n <= t < 0)
        i, op, opnd = t, "", b""
        body = cs[smp["cs_off"][r]: smp["cs_off"][r + 1]]
        for k in range(len(body) + 1):
            c = body[k: k + 1]
            if c and c not in b":Z+-*":
                opnd += c
                continue
            if opnd or not c:
                if op == ":":
                    i += int(opnd)
                elif op == "*":
                    i += 1
                elif op == "-":
                    i += len(opnd)
                elif op == "+":
                    ins += int(-n <= i < 0 and len(opnd) > 0)
            if c:
                op, opnd = c.decode(), b""
        down += int(dl > 0 and -n <= i < 0)
    return up, ins, down
