"""Multi-GPU pileup: reads sharded across GPUs, one global pileup.

Shards own CONTIGUOUS global read ranges in shard order (rank k holds the
k-th block of every sample's reads).  This preserves the one piece of the
reference that depends on read order: the slot layout at gaps that receive
both LEFT and RIGHT strings (processBaseString_leftIndel / _rightIndel,
mapped_paf_read_parser.py:37-72, driven in PAF first-occurrence order :292).
Everything else is an order-free integer tally.  See SURVEY.md 8(e).

Every shard runs the phases of include/mpc.h on its own reads.  Between the
phases it exchanges small per-gap / per-run arrays (no read data moves), four
collectives per step:

    after parse     OR      hasleft bitmap        (which gaps hold LEFT events)
    after index     GATHER  per-gap mixed RIGHT counts -> global run index space
    after tally     MAX     MAXR | M[:used] | RUN_R[:used] (RUN_R parked in M's
                            unused tail: one reduction), used = the runs in use
                            (G + all shards' mixed RIGHT events, read on the host
                            once per batch): longest RIGHT string at RIGHT-only
                            gaps, longest LEFT string per run, RIGHT string
                            closing each run
    after rows      SUM     rows                  (every shard's rows hold its own
                            reads' counts, odd positions included)

The depth difference array and the substitution tallies are never exchanged:
they are linear, so they reach the result through the rows SUM.  Layout and
consensus are then identical on every shard.  The protocol
is written once against an ``Exchange``: ``DistExchange`` is one shard per
process over torch.distributed (RCCL over xGMI on GPUs; gloo in the CPU
tests), ``LocalExchange`` drives several shards in one process (used by the
GPU parity test to check the sharded kernels bit-exactly against one GPU).
"""
import numpy as np

from . import engine as eng


class LocalExchange:
    """Collectives over a list of tensors that all live in this process (one per shard)."""

    def reduce(self, ts, op):
        acc = ts[0].clone()
        for t in ts[1:]:
            t = t.to(acc.device)
            if op == "sum":
                acc += t
            elif op == "max":
                acc = acc.maximum(t)
            elif op == "or":
                acc |= t
            else:
                raise ValueError(op)
        for t in ts:
            t.copy_(acc.to(t.device))

    def gather(self, ts, outs):
        """outs[i] (shape [n_shards * k]) <- concatenation of ts in shard order."""
        import torch
        for o in outs:
            o.copy_(torch.cat([t.to(o.device) for t in ts]))

    def max_int(self, xs):
        return [max(xs)] * len(xs)

    def sizes(self, ns):
        return list(ns)


class DistExchange:
    """One shard per process over a torch.distributed process group."""

    def __init__(self, group=None):
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        # RCCL ("nccl") works on device tensors in place; gloo (CPU tests, the
        # one-GPU rehearsal of N ranks) gets host copies of device tensors
        self.host_staged = dist.get_backend(group) != "nccl"

    def reduce(self, ts, op):
        (t,) = ts
        if self.host_staged and t.is_cuda:
            h = t.cpu()
            self.reduce([h], op)
            t.copy_(h)
            return
        d = self.dist
        if op == "sum":
            d.all_reduce(t, op=d.ReduceOp.SUM, group=self.group)
        elif op == "max":
            d.all_reduce(t, op=d.ReduceOp.MAX, group=self.group)
        elif op == "or":
            # RCCL has no bitwise reduction: gather the bitmaps, OR them as a tree
            # (a fresh output per call: one exchange may serve pipelines on several streams)
            st = self._gather_rows(t)
            k = self.world
            while k > 2:
                h = (k + 1) // 2  # rows [h, k) fold onto [0, k - h)
                st[: k - h] |= st[h:k]
                k = h
            if k == 2:
                import torch
                torch.bitwise_or(st[0], st[1], out=t)  # the last fold straight into t
            else:
                t.copy_(st[0])
        else:
            raise ValueError(op)

    def _gather_rows(self, t, out=None):
        """(world, len(t)) tensor of every rank's t, by one all_gather_into_tensor
        (straight into ``out`` when given; RCCL and gloo alike)."""
        import torch
        if out is None:
            out = torch.empty((self.world,) + tuple(t.shape), dtype=t.dtype, device=t.device)
        self.dist.all_gather_into_tensor(out.view(-1), t.contiguous(), group=self.group)
        return out

    def gather(self, ts, outs):
        (t,), (o,) = ts, outs
        if self.host_staged and (t.is_cuda or o.is_cuda):
            h = self._gather_rows(t.cpu())
            o.copy_(h.view(-1))
            return
        self._gather_rows(t, o.view(self.world, -1))

    def _ints(self, xs, op):
        import torch
        dev = "cuda" if self.dist.get_backend(self.group) == "nccl" else "cpu"
        if op == "max":
            t = torch.tensor(xs, dtype=torch.int64, device=dev)
            self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX, group=self.group)
            return [int(t.item())]
        t = torch.tensor(xs, dtype=torch.int64, device=dev)
        parts = [torch.empty_like(t) for _ in range(self.world)]
        self.dist.all_gather(parts, t, group=self.group)
        return [int(p.item()) for p in parts]

    def max_int(self, xs):
        return self._ints(xs, "max")

    def sizes(self, ns):
        return self._ints(ns, "gather")


def split_samples(samples, n_shards):
    """Per-shard sample lists: shard k gets the k-th contiguous block of every
    sample's reads (buffers are shared, offsets sliced)."""
    out = [[] for _ in range(n_shards)]
    for s in samples:
        n = len(s["tstart"])
        cuts = [n * k // n_shards for k in range(n_shards + 1)]
        for k in range(n_shards):
            a, b = cuts[k], cuts[k + 1]
            part = dict(s)
            for key in ("cs_off", "up_off", "down_off"):
                part[key] = np.asarray(s[key])[a: b + 1]
            for key in ("tstart", "aligned", "tend"):
                if key in s:
                    part[key] = np.asarray(s[key])[a:b]
            out[k].append(part)
    return out


def shard_layout(n_reads_per_shard):
    """(read_offset, n_reads_global) of every shard: shards are contiguous, in order."""
    offs = np.concatenate([[0], np.cumsum(n_reads_per_shard)]).astype(np.int64)
    return [int(o) for o in offs[:-1]], int(offs[-1])


def exchange_step(plans, ex, mdf, gtf, stream=None, used=None):
    """One global pileup over the shards in ``plans`` (all of this process's
    shards; with DistExchange exactly one).  Collective: every shard must call it.
    ``used`` (the runs in use, see below) is a property of the shards' reads:
    a caller that steps the same batches again passes the value this function
    returned for them, and the step then has no host synchronisation."""
    import torch
    i32 = torch.int32

    def each(phase, *args):
        for p in plans:
            p.phase(phase, stream, *args)

    each("parse")
    ex.reduce([p.buffer(eng.BUF_HASLEFT, i32) for p in plans], "or")
    each("index")
    ex.gather([p.buffer(eng.BUF_RIGHT_CNT, i32) for p in plans], [p.buffer(eng.BUF_RIGHT_CNT_ALL, i32) for p in plans])
    each("runs")
    each("tally")
    # MAXR (RIGHT-only gaps) and the USED runs of RUN_M / RUN_R: the run index
    # space is sized for every read being a mixed RIGHT event (runs_cap = global
    # reads + G: ~13 MB at C2 x 8 GPUs), the runs in use are G + all shards'
    # mixed RIGHT events (~35 k there).  One host read of that count (after the
    # gather it is on every shard), then two MAX reductions over the used parts
    # (MAXR and RUN_M are adjacent in the workspace)
    if used is None:
        used = int(plans[0].buffer(eng.BUF_MAXR, i32).numel()) + int(plans[0].buffer(eng.BUF_RIGHT_CNT_ALL, i32).sum())
    heads, tails, parked = [], [], []
    for p in plans:
        span = p.span(eng.BUF_MAXR, eng.BUF_RUN_M, i32)
        m = p.buffer(eng.BUF_RUN_M, i32)
        moff = (m.data_ptr() - span.data_ptr()) // 4
        rr = p.buffer(eng.BUF_RUN_R, i32)[:used]
        if 2 * used <= m.numel():
            # ONE max: RUN_R[:used] parked in RUN_M's unused tail [used, 2 used)
            # (no kernel reads runs >= used; the next clear zeroes it)
            m[used: 2 * used].copy_(rr)
            heads.append(span[: moff + 2 * used])
            parked.append((m[used: 2 * used], rr))
        else:
            heads.append(span[: moff + used])
            tails.append(rr)
    ex.reduce(heads, "max")
    if tails:
        ex.reduce(tails, "max")
    for src, dst in parked:
        dst.copy_(src)
    each("layout")
    each("rows")
    ex.reduce([p.buffer(eng.BUF_ROWS, i32) for p in plans], "sum")
    each("consensus", mdf, gtf)
    return used


class ShardedPileup:
    """Shards of one global pileup.  ``shards`` is a list of per-shard sample
    lists (every shard holds the same samples, i.e. the same references, and
    its own contiguous block of each sample's reads).

    With ``ex=None`` all shards live in this process (LocalExchange); with a
    DistExchange this process holds exactly one shard (``rank`` of the group).
    """

    def __init__(self, shards, devices, ex=None, row_cap=None, parse_cus=0):
        self.ex = ex or LocalExchange()
        local = len(shards)
        if isinstance(self.ex, DistExchange):
            assert local == 1, "one shard per process"
            ranks = [self.ex.rank]
            n_shards = self.ex.world
        else:
            ranks = list(range(local))
            n_shards = local
        n_local = [sum(len(s["tstart"]) for s in smp) for smp in shards]
        n_all = self.ex.sizes(n_local)
        offs, ng = shard_layout(n_all)
        self.batches = [eng.Batch(smp, device=dev, read_offset=offs[r], n_reads_global=ng, shard=r,
                                  n_shards=n_shards, parse_cus=parse_cus) for smp, dev, r in zip(shards, devices, ranks)]
        cap = row_cap or max(b.row_estimate() for b in self.batches)
        cap = self.ex.max_int([cap] * local)[0] if isinstance(self.ex, DistExchange) else cap
        self.plans = [eng.Plan(b, cap) for b in self.batches]
        self._sized = False
        # runs in use, read back once: valid for THESE batches only -- the
        # batches are fixed for the object's lifetime (mpc_plan_set_input is
        # never called on them); rebind() resets it
        self._used = None

    def rebind(self):
        """Forget the cached run count (call after changing any shard's inputs
        in place): the next step re-reads it before the run-array MAX."""
        self._used = None
        self._sized = False

    # bench.py interface (one local shard)
    @property
    def batch(self):
        return self.batches[0]

    @property
    def plan(self):
        return self.plans[0]

    def step(self, mdf, gtf, stream=None):
        # the runs in use depend only on the reads: read back once, reused by
        # later steps over the same batches (no host sync inside a step)
        used = exchange_step(self.plans, self.ex, mdf, gtf, stream, self._used)
        if not self._sized:
            # the layout (and so the row count) is identical on every shard
            st = self.plans[0].status()
            flags = int(st[eng.MPC_ST_FLAGS])
            flags = self.ex.max_int([flags] * len(self.plans))[0] if isinstance(self.ex, DistExchange) else flags
            if flags & eng.DE_CAPACITY:
                need = int(st[eng.MPC_ST_ROWS_NEEDED]) + 16
                self.plans = [eng.Plan(b, need) for b in self.batches]
                used = exchange_step(self.plans, self.ex, mdf, gtf, stream)
            self._sized = True
            self._used = used

    def check(self):
        for p in self.plans:
            st = p.status()
            if int(st[eng.MPC_ST_FLAGS]):
                raise eng.DataError(int(st[eng.MPC_ST_FLAGS]), int(st[eng.MPC_ST_FIRST_READ]))

    def fetch(self):
        return self.plans[0].fetch()
