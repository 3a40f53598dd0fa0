"""The multi-GPU protocol with REAL HIP plans across processes.

Two / three fresh processes share cuda:0 (RCCL needs one GPU per rank, so the
ranks exchange over gloo with host-staged tensors: dist.DistExchange), each
generates only its contiguous slice of one global read set (Synth(reads=...),
exactly as bench.py --gpus N does), runs ShardedPileup over its own plan, and
returns its fetched calls.  Every rank must hold the single-pileup result of
the whole read set, bit-exact with the C oracle -- including the order-dependent
slot layout at gaps with both LEFT and RIGHT events
(mapped_paf_read_parser.py:37-72 in the read order of :292).
"""
import importlib
import os
import socket

import pytest
import torch.multiprocessing as mp

import depth_util as du

pytestmark = pytest.mark.gpu

SPECS = {
    "c2like": dict(n=2686, n_reads=24_000, profile="default", seed=2, frac_partial=0.05),
    # >= 250k reads per strand over 2 processes: 125k reads per rank and strand
    "c2_250k": dict(n=2686, n_reads=250_000, profile="default", seed=2, frac_partial=0.02),
    "partial_indel": dict(n=900, n_reads=6_000, profile="indel", seed=71, frac_partial=0.5, flank=(0, 60),
                          ins_len=(1, 8), del_len=(1, 6)),
}


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, spec_name, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        import torch
        import torch.distributed as tdist
        torch.cuda.set_device(0)
        tdist.init_process_group("gloo", rank=rank, world_size=world)
        try:
            pkg = importlib.import_module("minion-plasmid-consensus_amd")
            dmod = importlib.import_module("minion-plasmid-consensus_amd.dist")
            spec = SPECS[spec_name]
            n = spec["n_reads"]
            a, b = n * rank // world, n * (rank + 1) // world
            syn = pkg.synth.Synth(reads=(a, b), **spec)
            samples = [syn.sample(0), syn.sample(1)]
            sp = dmod.ShardedPileup([samples], [0], ex=dmod.DistExchange())
            out = []
            for mdf, gtf in ((-1.0, 1.0), (0.1, 5.0)):
                sp.step(mdf, gtf)
                sp.check()
                out.append([{k: v for k, v in r.items()} for r in sp.fetch()])
            q.put((rank, out, None))
        finally:
            tdist.destroy_process_group()
    except Exception as e:  # reported to the parent
        q.put((rank, None, repr(e)))


@pytest.mark.timeout(300)
@pytest.mark.parametrize("spec_name,world", [("c2like", 2), ("partial_indel", 3), ("c2_250k", 2)])
def test_dist_exchange_real_plans(pkg, spec_name, world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, spec_name, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = sorted((q.get(timeout=240) for _ in range(world)), key=lambda x: x[0])
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for rank, _, err in res:
        assert err is None, (rank, err)
    for p in procs:
        assert p.exitcode == 0
    syn = pkg.synth.Synth(**SPECS[spec_name])
    samples = [syn.sample(0), syn.sample(1)]
    full = du.oracle_many(samples, -1.0, 1.0)
    for rank, out, _ in res:
        for (mdf, gtf), got in zip(((-1.0, 1.0), (0.1, 5.0)), out):
            for s, (g, f) in enumerate(zip(got, full)):
                du.compare(g, du.derive(f, mdf, gtf), (spec_name, world, rank, s, mdf))


@pytest.mark.timeout(900)
def test_c3_eight_shards_in_process(pkg):
    """BASELINE configs[2] (C3: 10 kb, 1M reads, sense) exactly as bench.py
    --gpus 8 splits it -- 8 contiguous shards of ONE global read order -- with
    the 8 shards' plans on this GPU and the exchanges in-process
    (LocalExchange).  Every shard must end with the single-pileup result,
    bit-exact with the C oracle, at full pileup and at 0.1 / 5.  The run replay
    at mixed gaps depends on the global read order (mapped_paf_read_parser.py:292,
    :37-72), so this pins the shard seams at size."""
    bench = importlib.import_module("bench")
    dist = importlib.import_module("minion-plasmid-consensus_amd.dist")
    samples, total = bench.shard_samples(pkg, "c3", 0, 1)
    assert total == 1_000_000 and len(samples) == 1
    full = du.oracle_many(samples, -1.0, 1.0)
    sp = dist.ShardedPileup(dist.split_samples(samples, 8), [0] * 8)
    for mdf, gtf in ((-1.0, 1.0), (0.1, 5.0)):
        sp.step(mdf, gtf)
        sp.check()
        for k, plan in enumerate(sp.plans):
            for s, (got, f) in enumerate(zip(plan.fetch(), full)):
                du.compare(got, du.derive(f, mdf, gtf), ("c3x8", k, s, mdf))
    del sp


def _nccl_worker(port, q):
    """ONE rank on cuda:0 over RCCL ("nccl"): two ShardedPileups in flight on
    two streams, each with its OWN communicator (dist.new_group per pipeline,
    exactly as bench.py builds them), stepped eagerly and then replayed from
    one HIP graph per pipeline (bench.py's default at N > 1 over RCCL)."""
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        import torch
        import torch.distributed as tdist
        torch.cuda.set_device(0)
        tdist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
        try:
            pkg = importlib.import_module("minion-plasmid-consensus_amd")
            dmod = importlib.import_module("minion-plasmid-consensus_amd.dist")
            bench = importlib.import_module("bench")
            samples, _ = bench.shard_samples(pkg, "c2", 0, 1)
            groups = [tdist.new_group([0]) for _ in range(2)]
            exs = [dmod.DistExchange(g) for g in groups]
            assert not any(ex.host_staged for ex in exs)  # device tensors in place: the RCCL branches
            sps = [dmod.ShardedPileup([samples], [0], ex=ex) for ex in exs]
            streams = [torch.cuda.current_stream(), torch.cuda.Stream()]
            out = []
            for mdf, gtf in ((-1.0, 1.0), (0.1, 5.0)):
                for rep in range(2):  # the second pass runs without host syncs (cached run count)
                    for k in (0, 1):
                        with torch.cuda.stream(streams[k]):
                            sps[k].step(mdf, gtf)
                torch.cuda.synchronize()
                for k in (0, 1):
                    sps[k].check()
                    out.append((mdf, gtf, k, "eager", [dict(r) for r in sps[k].fetch()]))
            # graph replay, as bench.py captures it: warm step on the capture
            # stream, then the captured step; replayed twice on the pipelines' streams
            mdf, gtf = 0.1, 5.0
            graphs = []
            for sp in sps:
                g = torch.cuda.CUDAGraph()
                cap = torch.cuda.Stream()
                with torch.cuda.stream(cap):
                    sp.step(mdf, gtf)
                    cap.synchronize()
                    with torch.cuda.graph(g, stream=cap):
                        sp.step(mdf, gtf)
                graphs.append(g)
            torch.cuda.synchronize()
            # a full-pileup step in between, so the replay must rewrite every output
            for k in (0, 1):
                sps[k].step(-1.0, 1.0)
            torch.cuda.synchronize()
            for rep in range(2):
                for k in (0, 1):
                    with torch.cuda.stream(streams[k]):
                        graphs[k].replay()
            torch.cuda.synchronize()
            for k in (0, 1):
                sps[k].check()
                out.append((mdf, gtf, k, "graph", [dict(r) for r in sps[k].fetch()]))
            del graphs
            q.put((out, None))
        finally:
            tdist.destroy_process_group()
    except Exception as e:  # reported to the parent
        import traceback
        q.put((None, traceback.format_exc() + repr(e)))


@pytest.mark.timeout(600)
def test_rccl_world1_two_pipelines(pkg):
    """The nccl (RCCL) branch of dist.DistExchange executed on hardware: a
    world-size-1 process group on cuda:0 (init_process_group("nccl",
    device_id=...)), C2 at full size (BASELINE configs[1]), two pipelines in
    flight, each on its own communicator (dist.new_group, as bench.py builds
    them), stepped eagerly and replayed from HIP graphs.  Every call of both
    pipelines must equal the C oracle's at full pileup and at 0.1 / 5 (VERDICT
    r03 item 3)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_nccl_worker, args=(_free_port(), q))
    p.start()
    try:
        out, err = q.get(timeout=540)
    finally:
        p.join(timeout=60)
        if p.is_alive():
            p.kill()
    assert err is None, err
    assert p.exitcode == 0
    bench = importlib.import_module("bench")
    samples, _ = bench.shard_samples(pkg, "c2", 0, 1)
    full = du.oracle_many(samples, -1.0, 1.0)
    assert len(out) == 6
    for mdf, gtf, k, how, got in out:
        for s, (g, f) in enumerate(zip(got, full)):
            du.compare(g, du.derive(f, mdf, gtf), ("rccl1", how, k, s, mdf))


@pytest.mark.timeout(600)
def test_bench_self_launch_two_ranks(tmp_path):
    """``python bench.py --gpus 2`` with no launcher starts 2 rank processes
    itself (torch.distributed.run as a child) -- here rehearsed on one GPU over
    gloo -- and rank 0's JSON line reports n_gpus == 2."""
    import json
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["MPC_DIST_BACKEND"] = "gloo"
    cmd = [sys.executable, os.path.join(repo, "bench.py"), "--gpus", "2", "--config", "c2", "--steps", "3",
           "--warmup", "1", "--kernel-reps", "2", "--inflight", "2", "--hbm-config", ""]
    p = subprocess.run(cmd, env=env, cwd=str(tmp_path), capture_output=True, text=True, timeout=540)
    assert p.returncode == 0, p.stderr[-4000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-4000:]
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2
    assert rec["config"]["parallelism"] == "read-shardx2"
    assert rec["config"]["process_group"] == "gloo"
    assert rec["config"]["global_reads_per_sample"] == 200_000  # weak scaling: 2 x 100k
    assert rec["value"] > 0
    # the N=2 line carries the per-rank K_parse HBM traffic
    # rocprofv3 measured on a rank's shard of the 2-shard plan
    assert rec["roofline"]["traffic"] is not None and rec["roofline"]["traffic"] > 0
    assert rec["roofline"]["traffic_record"] == "profiles/pmc_traffic_c2_w2.json"
    assert rec["config"]["batches_in_flight"] == 2  # (--inflight 2 here; the N > 1 default is 2 as well)
