"""The N>1 exchange protocol on the CPU (gloo, world size 2).

The HIP phases need a GPU, so the plans here are stand-ins that expose the
exchange buffers of include/mpc.h as CPU tensors and record the phase order.
What is checked is exactly the multi-GPU plumbing of dist.exchange_step: the
phase order, which buffer is combined with which reduction, and that the
torch.distributed exchange (DistExchange over gloo) gives the same bytes as
the in-process LocalExchange.  The sharded kernels themselves are checked
bit-exactly on the GPU (test_gpu_parity.py::test_sharded_*).
"""
import importlib
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

G = 37  # gaps
ROWS = 23


def _mod():
    return importlib.import_module("minion-plasmid-consensus_amd.dist"), importlib.import_module(
        "minion-plasmid-consensus_amd.engine")


class FakePlan:
    """Exchange buffers of one shard, seeded per shard; phases are recorded."""

    def __init__(self, shard, n_shards, mlen=G + 11):
        _, eng = _mod()
        rng = np.random.default_rng(1000 + shard)
        i = lambda *shape, hi=1000: torch.from_numpy(rng.integers(0, hi, size=shape).astype(np.int32))
        # MAXR, RUN_M, RUN_R: one workspace span with padding between them (include/mpc.h);
        # mlen >= 2 x the runs in use: RUN_R is reduced parked in RUN_M's tail (one MAX)
        self.mlen = mlen
        self.mx = i(G + 5 + mlen + 3 + mlen)
        a, b = G + 5, G + 5 + mlen + 3
        self.buf = {
            eng.BUF_HASLEFT: i((G + 31) // 32 + 1, hi=2 ** 30),
            eng.BUF_DIFF: i(G), eng.BUF_SUB: i(4 * G),
            # a few mixed RIGHT events: the runs in use (G + their sum) stop short of the run buffers' end
            eng.BUF_RIGHT_CNT: i(G, hi=2) * (torch.arange(G) < 3).to(torch.int32),
            eng.BUF_RIGHT_CNT_ALL: torch.zeros(n_shards * G, dtype=torch.int32),
            eng.BUF_MAXR: self.mx[:G], eng.BUF_RUN_M: self.mx[a:a + mlen], eng.BUF_RUN_R: self.mx[b:b + mlen],
            eng.BUF_ROWS: i(4 * ROWS),
        }
        self.initial = {k: v.clone() for k, v in self.buf.items()}
        self.log = []

    def phase(self, name, stream=None, *args):
        self.log.append((name,) + tuple(args))

    def buffer(self, which, dtype):
        return self.buf[which]

    def span(self, first, last, dtype):
        _, eng = _mod()
        assert (first, last) == (eng.BUF_MAXR, eng.BUF_RUN_M)
        return self.mx[: G + 5 + self.mlen]


def expected(n_shards, mlen=G + 11):
    """(combined buffers, the combined used head of RUN_M / RUN_R, the runs in use)."""
    _, eng = _mod()
    plans = [FakePlan(k, n_shards, mlen) for k in range(n_shards)]
    init = [p.initial for p in plans]
    out = {}
    # DIFF / SUB stay per shard (every shard's rows carry its own odd-position counts)
    for b, op in ((eng.BUF_HASLEFT, "or"), (eng.BUF_MAXR, "max"), (eng.BUF_ROWS, "sum")):
        acc = init[0][b].clone()
        for x in init[1:]:
            acc = acc + x[b] if op == "sum" else (acc.maximum(x[b]) if op == "max" else acc | x[b])
        out[b] = acc
    out[eng.BUF_RIGHT_CNT_ALL] = torch.cat([x[eng.BUF_RIGHT_CNT] for x in init])
    # runs in use: G + all shards' mixed RIGHT events; the MAX covers only them
    used = G + sum(int(x[eng.BUF_RIGHT_CNT].sum()) for x in init)
    assert used < G + 11
    heads = {}
    for b in (eng.BUF_RUN_M, eng.BUF_RUN_R):
        acc = init[0][b][:used].clone()
        for x in init[1:]:
            acc = acc.maximum(x[b][:used])
        heads[b] = acc
    return out, heads, used


def _check(p, exp):
    _, eng = _mod()
    full, heads, used = exp
    ok = all(torch.equal(p.buf[b], v) for b, v in full.items())
    for b, v in heads.items():
        ok = ok and torch.equal(p.buf[b][:used], v)
        if b == eng.BUF_RUN_M and 2 * used <= p.mlen:  # RUN_R's reduced head parked behind the used runs
            ok = ok and torch.equal(p.buf[b][used: 2 * used], heads[eng.BUF_RUN_R])
            ok = ok and torch.equal(p.buf[b][2 * used:], p.initial[b][2 * used:])
        else:
            ok = ok and torch.equal(p.buf[b][used:], p.initial[b][used:])
    return ok


PHASES = ["parse", "index", "runs", "tally", "layout", "rows", "consensus"]


@pytest.mark.parametrize("mlen", [G + 11, 3 * G])  # two MAX reductions / one (RUN_R parked in RUN_M)
def test_local_exchange_combines(mlen):
    dist, eng = _mod()
    plans = [FakePlan(k, 3, mlen) for k in range(3)]
    dist.exchange_step(plans, dist.LocalExchange(), 0.1, 5.0)
    exp = expected(3, mlen)
    for p in plans:
        assert [x[0] for x in p.log] == PHASES
        assert p.log[-1] == ("consensus", 0.1, 5.0)
        assert _check(p, exp)
        for b in (eng.BUF_RIGHT_CNT, eng.BUF_DIFF, eng.BUF_SUB):  # per-shard buffers untouched
            assert torch.equal(p.buf[b], p.initial[b]), b


def test_shard_layout_and_split():
    dist, _ = _mod()
    offs, ng = dist.shard_layout([5, 0, 7])
    assert offs == [0, 5, 5] and ng == 12
    s = dict(ref=np.zeros(3, np.uint8), cs=np.zeros(10, np.uint8), cs_off=np.arange(11), up=np.zeros(0, np.uint8),
             up_off=np.zeros(11, np.int64), down=np.zeros(0, np.uint8), down_off=np.zeros(11, np.int64),
             tstart=np.arange(10), aligned=np.ones(10))
    parts = dist.split_samples([s, s], 3)
    assert [len(p[0]["tstart"]) for p in parts] == [3, 3, 4]
    assert np.array_equal(np.concatenate([p[1]["tstart"] for p in parts]), s["tstart"])
    for p in parts:
        assert len(p[0]["cs_off"]) == len(p[0]["tstart"]) + 1


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as tdist
    tdist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dist, eng = _mod()
        ex = dist.DistExchange()
        plan = FakePlan(rank, world)
        dist.exchange_step([plan], ex, 0.5, 2.5)
        exp = expected(world)
        ok = [x[0] for x in plan.log] == PHASES and _check(plan, exp)
        sizes = ex.sizes([10 + rank])
        mx = ex.max_int([rank * 7])
        q.put((rank, bool(ok), sizes, mx))
    finally:
        tdist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_dist_exchange_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, ok, sizes, mx in res:
        assert ok, rank
        assert sizes == [10 + r for r in range(world)]
        assert mx == [7 * (world - 1)]
