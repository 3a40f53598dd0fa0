#!/usr/bin/env python3
"""Benchmark: aligned bases/s of pileup + consensus on MI355X (BASELINE.json metric).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2]

A step = one full pass of the hot path (Steps 4-6 of the reference: cs parse
-> pileup -> consensus calls) over one batch of synthetic, seeded,
device-resident input.  At N=1 the workload is BASELINE.json configs[1] (C2:
pUC19-size 2,686 bp plasmid, 100k reads, sense + antisense in one launch).

Multi-GPU (torch.distributed.run, one rank per GPU, RCCL): every config is ONE
global pileup over ONE read set (same reference, same seed); rank k holds the
k-th contiguous slice of the global read order (Synth(reads=(a, b)) generates
exactly those reads of the full set) and the ranks exchange the small per-gap
/ per-run arrays of minion-plasmid-consensus_amd/dist.py.
  c1, c2, c4   weak scaling: the global set has N x (reads per GPU) reads
  c3           strong scaling: 1M reads in total, N slices (BASELINE configs[2])
  c5           sample-partitioned replicas: 12 plasmids per GPU, no collective

Batches in flight (--inflight R, default per config: C1 4, C2 3, else 2): R independent pipelines (each its
own device copy of the batch and its own workspace) on R streams, taken in
turn, so one batch's latency-bound post-parse chain overlaps the next batch's
parse -- a stream of plasmid batches as a sequencing run produces them.  Every
step is still one full pass of the hot path over one batch; value = aligned
bases of all K steps / wall time.  --inflight 1 runs them one after another.

Output: one JSON line (rank 0) with the contract fields plus
  roofline      the dominant kernel (K_parse) vs the HBM roofline: algorithmic
                bytes (sum of cs bytes + 24 B per read) / its mean
                duration measured here with HIP events on the launch stream;
                traffic = HBM bytes per launch from rocprofv3 PMC passes
                (profiles/pmc_traffic_<config>.json, scripts/traffic.py)
  cpu_baseline  the C restatement of the reference (oracle/, "port") timed on
                this host on a bounded read sample, 1 thread (rank 0, N=1 only),
                and under "reference" the reference script itself timed in the
                build container (profiles/ref_cpu_baseline.json,
                scripts/time_reference.py)
  e2e           (N=1, every config) the drop-in CLI on files of the same
                workload, all of the GPU's jobs in one call (c5: 24 jobs, 72
                output files): ingest + H2D + kernels + D2H + writers, wall
                clock, with the phase split
"""
import argparse
import contextlib
import importlib
import io
import json
import os
import shutil
import sys
import tempfile
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "aligned bases/sec pileup+consensus (1/2/4/8 GPU) and % HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)

CONFIGS = {
    # name: (n, reads per sample, per-GPU (weak) or total (strong), profile, seed, antisense, description)
    "c2": (2686, 100_000, "weak", "default", 2, True,
           "C2 (BASELINE configs[1]): pUC19-size 2,686 bp plasmid, 100k reads per GPU, sense+antisense pileup"),
    "c1": (5000, 20_000, "weak", "default", 1, False,
           "C1 (BASELINE configs[0]): 5 kb plasmid, 20k reads per GPU, sense only"),
    "c3": (10_000, 1_000_000, "strong", "default", 3, False,
           "C3 (BASELINE configs[2]): 10 kb plasmid, 1M reads in total sharded over the GPUs, sense"),
    "c4": (10_000, 100_000, "weak", "indel", 4, True,
           "C4 (BASELINE configs[3]): 10 kb, 100k reads per GPU, indel-heavy 1/5/5 %, sense+antisense"),
    "c5": (30_000, 10_000, "weak", "default", 5000, True,
           "C5 (BASELINE configs[4]): 30 kb BAC-size constructs, 12 plasmids x 10k reads per GPU "
           "(96 over 8 GPUs), sense+antisense, sample-partitioned"),
}
C5_PER_GPU = 12
# batches in flight per config, and the CUs the parse grid is sized for with
# them (20-step runs): C2 3 / 192 (2 / 160 200 us per step, 3 / 192 182.5 us,
# 4 / 128 183 us; profiles/r04_experiments/c2_batches_in_flight.txt), C1
# 4 / 96 (2 / 128 85 us, 3 / 128 69 us, 4 / 96 62 us), C3-C5 2 (3 is no
# faster: batches_in_flight_c1_c3_c4_c5.txt; their CUs:
# profiles/r03_experiments/parse_cus_inflight.txt)
INFLIGHT = {"c1": 4, "c2": 3, "c3": 2, "c4": 2, "c5": 2}
PARSE_CUS_INFLIGHT = {"c1": 96, "c2": 192, "c3": 224, "c4": 224, "c5": 192}
# pipelines in flight per rank at world size > 1 (2 compute + 2 communicator
# streams = the 4 hardware queues a process gets)
MAX_PIPELINES_DIST = 2
PORT_SAMPLE_BASES = 2_500_000_000  # bound of the live CPU-port timing (~6 s of C at ~4e8 b/s)
E2E_CONFIGS = ("c1", "c2", "c3", "c4", "c5")


def shard_samples(pkg, cfg, rank, world):
    """This rank's samples: its slice of the global read set (c1-c4), or its
    plasmids (c5).  Returns (samples, global reads per sample)."""
    n, reads, scaling, profile, seed, antisense, _ = CONFIGS[cfg]
    strands = range(2 if antisense else 1)
    if cfg == "c5":
        samples = []
        for k in range(C5_PER_GPU):
            syn = pkg.synth.Synth(n=n, n_reads=reads, profile=profile, seed=seed + C5_PER_GPU * rank + k,
                                  antisense=antisense)
            samples += [syn.sample(s) for s in strands]
        return samples, reads
    total = reads * world if scaling == "weak" else reads
    a, b = total * rank // world, total * (rank + 1) // world
    syn = pkg.synth.Synth(n=n, n_reads=total, profile=profile, seed=seed, antisense=antisense, reads=(a, b))
    return [syn.sample(s) for s in strands], total


def port_baseline(samples, mdf, gtf, cfg):
    """The oracle's C restatement over the first reads of every sample, at most
    PORT_SAMPLE_BASES aligned bases in total (1 thread)."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle  # CPU checker: timed here as the baseline, never on the product path
    budget = PORT_SAMPLE_BASES // len(samples)
    cb, nr, tot_reads, t = 0, 0, 0, 0.0
    for s in samples:
        al = np.asarray(s["aligned"], dtype=np.int64)
        k = int(np.searchsorted(np.cumsum(al), budget, side="right")) if al.sum() > budget else len(al)
        k = max(1, min(k, len(al)))
        c0 = time.perf_counter()
        oracle.run_packed(s["ref"], s["cs"], s["cs_off"][: k + 1], s["tstart"][:k], s["up"], s["up_off"][: k + 1],
                          s["down"], s["down_off"][: k + 1], mdf, gtf)
        t += time.perf_counter() - c0
        cb += int(al[:k].sum())
        nr += k
        tot_reads += len(al)
    frac = nr / max(1, tot_reads)
    return {"value": cb / t, "unit": "aligned bases/s", "cores": 1, "kind": "port",
            "sample": f"{cfg}: first {nr} of {tot_reads} reads ({100 * frac:.3g} %) over {len(samples)} sample(s), "
                      f"{cb} aligned bases through oracle/mpc_oracle.c, 1 thread, {t:.2f} s"}


def reference_record(cfg):
    try:
        rec = json.load(open(os.path.join(REPO, "profiles", "ref_cpu_baseline.json")))
    except (OSError, ValueError):
        return None
    r = rec.get("configs", {}).get(cfg)
    if r is not None:
        r = dict(r, host=rec.get("host"))
    return r


def e2e_cli(pkg, cfg, reps=2):
    """Wall time of the drop-in CLI on files of this config, all of a GPU's jobs
    in ONE CLI call (c2/c4: --also for the antisense strand; c5: --job per
    plasmid and strand, 12 plasmids = 24 jobs = 72 output files): native ingest
    + H2D + plan + kernels + D2H + native writers.  Returns a dict with the
    phase split (ingest / device / write) of the best repetition."""
    cli = importlib.import_module("minion-plasmid-consensus_amd.mapped_paf_read_parser")
    n, reads, _, profile, seed, antisense, _ = CONFIGS[cfg]
    tmp = tempfile.mkdtemp(prefix="mpc_e2e_")
    try:
        p = lambda f: os.path.join(tmp, f)
        plasmids = C5_PER_GPU if cfg == "c5" else 1
        argv, aligned, n_files = [], 0, 0
        for k in range(plasmids):
            syn = pkg.synth.Synth(n=n, n_reads=reads, profile=profile, seed=seed + k, antisense=antisense)
            aligned += int(sum(int(syn.sample(s)["aligned"].sum()) for s in range(2 if antisense else 1)))
            syn.write_files(p(f"ref{k}.fa"), p(f"reads{k}.fa"), p(f"s0_{k}.paf"), p(f"ref{k}_as.fa") if antisense else None,
                            p(f"s1_{k}.paf") if antisense else None)
            del syn
            strands = [(p(f"ref{k}.fa"), p(f"s0_{k}.paf"))] + ([(p(f"ref{k}_as.fa"), p(f"s1_{k}.paf"))] if antisense else [])
            for s, (ref, paf) in enumerate(strands):
                argv += ["--job", ref, paf, p(f"reads{k}.fa"), p(f"c{k}_{s}.fa"), p(f"ch{k}_{s}.tsv"), p(f"acc{k}_{s}.tsv")]
                n_files += 3
        argv += ["--min_depth_factor", "0.1", "--global_threshold_factor", "5"]
        in_bytes = sum(os.path.getsize(p(f)) for f in os.listdir(tmp))
        runs = []
        for _ in range(reps):
            sink = io.StringIO()
            tm = {}
            t0 = time.perf_counter()
            with contextlib.redirect_stdout(sink):
                rc = cli.main(argv, timings=tm)
            tm["wall"] = time.perf_counter() - t0
            runs.append(tm)
            if rc != 0:
                raise RuntimeError(f"CLI exit {rc}")
        best = min(runs, key=lambda r: r["wall"])
        out_bytes = sum(os.path.getsize(p(f)) for f in os.listdir(tmp) if f.startswith(("c", "acc")) and "_" in f)
        return {"value": aligned / best["wall"], "unit": "aligned bases/s", "wall_s": best["wall"],
                "wall_s_first": runs[0]["wall"], "aligned_bases": aligned, "input_bytes": in_bytes,
                "output_files": n_files, "output_bytes": out_bytes,
                "phases_s": {k: round(best[k], 4) for k in ("setup", "ingest", "device", "write", "main") if k in best},
                "write_frac": best["write"] / best["wall"],
                "what": f"{cfg} files, {len(argv) // 7} job(s) in ONE CLI call (--job each), {n_files} output files; "
                        "CLI main(): native ingest of ref/PAF/reads FASTA + H2D + plan + kernels + D2H + "
                        "writers of the output files; best of %d (first includes allocations)" % reps}
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


# what bounds K_parse by its counters (profiles/r03_stalls_*)
LIMITER = ("dependency latency of the per-round chain (dependent LDS round trips and a DPP scan per 64 units): "
           "waves issue 36 %, wait on s_waitcnt 35 %, dependency-stalled 29 % of their cycles; VALU at 35-60 % of "
           "its measured 4-wave rate (profiles/r03_stalls_c2_final, profiles/r03_micro); window + decode work "
           "(no effects) is 65-71 % of the kernel (profiles/r04_experiments/kparse_tokenize_only.txt; DESIGN.md §3)")


# roofline.bound: what limits K_parse as measured (its HBM fraction is still
# reported against the 8 TB/s peak): latency of the per-round dependency chain
ROOF_BOUND = "latency"


def batch_l3_resident(cfg):
    """Whether the kernel's input (cs + records) fits the 256 MiB Infinity Cache
    between launches: then the FETCH counters and the achieved rate include L3 hits."""
    n, reads, _, _, _, anti, _ = CONFIGS[cfg]
    per_read = {"c1": 0.12, "c2": 0.12, "c3": 0.12, "c4": 0.53, "c5": 0.12}[cfg] * n + 24
    samples = (C5_PER_GPU if cfg == "c5" else 1) * (2 if anti else 1)
    return bool(per_read * reads * samples < 200e6)


def kernel_roofline(pkg, eng, cfg, reps, torch):
    """K_parse alone on ``cfg`` (device-resident), HIP events on its stream."""
    samples, _ = shard_samples(pkg, cfg, 0, 1)
    runner = eng.Runner(samples)
    runner.step(0.1, 5.0)
    runner.check()
    plan, batch = runner.plan, runner.batch
    stream = torch.cuda.current_stream()
    for _ in range(2):
        plan.profile_kernel(eng.K_PARSE)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record(stream)
        plan.profile_kernel(eng.K_PARSE)
        b.record(stream)
    torch.cuda.synchronize()
    k_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    alg = batch.cs_bytes + 24 * batch.n_reads
    achieved = alg / (k_ms * 1e-3) / 1e9
    traffic = None
    try:
        tr = json.load(open(os.path.join(REPO, "profiles", f"pmc_traffic_{cfg}.json")))
        if tr.get("config") == cfg and tr.get("kernel") == "K_parse":
            traffic = tr.get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        pass
    out = {"config": cfg, "bound": ROOF_BOUND, "kernel": "K_parse", "achieved": achieved, "peak": HBM_PEAK_GBS,
           "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "alg_bytes_per_launch": alg,
           "mean_launch_us": k_ms * 1e3, "aligned_bases_per_launch": batch.aligned_bases,
           "input_l3_resident": batch_l3_resident(cfg), "parse_geometry": plan.info()}
    del runner, plan, batch
    torch.cuda.empty_cache()
    return out


def traffic_record(cfg, world):
    """(HBM bytes per K_parse launch, record file) from rocprofv3 PMC passes for
    this config at this GPU count: profiles/pmc_traffic_<cfg>.json (N = 1) or
    pmc_traffic_<cfg>_w<N>.json (one rank's shard of the N-shard plan measured on
    one GPU, scripts/shard_traffic.sh).  C5 runs replicas (every GPU the N = 1
    plan over its own plasmids): its N = 1 record.  (None, None) if absent."""
    names = [f"pmc_traffic_{cfg}.json"] if world == 1 else [f"pmc_traffic_{cfg}_w{world}.json"]
    if world > 1 and cfg == "c5":
        names.append(f"pmc_traffic_{cfg}.json")
    for nm in names:
        try:
            tr = json.load(open(os.path.join(REPO, "profiles", nm)))
        except (OSError, ValueError):
            continue
        n_ok = tr.get("n_gpus", 1) == world or (cfg == "c5" and tr.get("n_gpus", 1) == 1)
        if tr.get("config") == cfg and tr.get("kernel") == "K_parse" and n_ok:
            return tr.get("hbm_bytes_per_launch"), "profiles/" + nm
    return None, None


def launch_ranks(n, argv):
    """``bench.py --gpus N`` (N > 1) started WITHOUT a launcher: run the same
    command as N rank processes (one per GPU) under torch.distributed.run, as a
    child of this process, and return its exit status.  This process never
    touches the GPU (nothing HIP is initialised before the children start; the
    JSON line is printed by rank 0 of the children)."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on this pool (RCCL)
    return subprocess.call(cmd, env=env)


def world_from_env(gpus):
    """(world, launched): the rank count of this run.  Under a launcher it is
    WORLD_SIZE, which must equal ``--gpus`` when that is given; without one it
    is 1 (``--gpus N > 1`` self-launches first, see launch_ranks)."""
    if "WORLD_SIZE" in os.environ:
        world = int(os.environ["WORLD_SIZE"])
        if gpus is not None and gpus != world:
            raise SystemExit(f"bench.py: --gpus {gpus} but the launcher started WORLD_SIZE={world} ranks")
        return world, True
    if gpus is not None and gpus < 1:
        raise SystemExit(f"bench.py: --gpus must be >= 1, got {gpus}")
    return 1, False


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (one rank each); without a launcher, N > 1 starts N ranks itself "
                         "(torch.distributed.run); under one it must equal WORLD_SIZE")
    # 200 steps: with R batches in flight the timed region starts with the
    # pipelines empty and ends draining them; at 20 steps that fill / drain was
    # ~9 % of C2's wall (175 vs 159 us per step, profiles/r06_experiments/
    # c2_parse_cus_steps.txt) -- a sequencing run streams far more batches
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--kernel-reps", type=int, default=20)
    ap.add_argument("--inflight", type=int, default=None,
                    help="batches in flight (independent pipelines on their own streams, taken in turn; "
                         "default per config: INFLIGHT)")
    ap.add_argument("--parse-cus", type=int, default=None,
                    help="CUs the parse grid is sized for with batches in flight (default: per config)")
    ap.add_argument("--dist", action="store_true",
                    help="take the distributed path (process group + dist.DistExchange) even at WORLD_SIZE=1")
    ap.add_argument("--graph", choices=("auto", "on", "off"), default="auto", nargs="?", const="on",
                    help="distributed path: replay every pipeline's step from a HIP graph (no host dispatch); "
                         "auto = on for RCCL at world size > 1; a bare --graph = on")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true")
    ap.add_argument("--hbm-config", default="c3", type=lambda s: s.strip().lower(),
                    help="also time K_parse on this (L3-exceeding) config for the HBM roofline; "
                         "'' or 'none' to skip")
    argv = sys.argv[1:]
    args = ap.parse_args(argv)
    if args.hbm_config in ("", "none"):
        args.hbm_config = ""
    elif args.hbm_config not in CONFIGS:
        ap.error(f"--hbm-config {args.hbm_config!r}: not one of {sorted(CONFIGS)} (or '' / none)")

    world, launched = world_from_env(args.gpus)
    if not launched and (args.gpus or 1) > 1:
        sys.exit(launch_ranks(args.gpus, argv))

    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one rank per GPU; the modulo only matters for rehearsals with more ranks than GPUs
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    # RCCL ("nccl") over xGMI; MPC_DIST_BACKEND=gloo rehearses the N>1 path on one GPU
    backend = os.environ.get("MPC_DIST_BACKEND", "nccl")
    use_dist = world > 1 or args.dist
    if use_dist:
        os.environ.setdefault("MASTER_PORT", "29517")
        os.environ.setdefault("RANK", str(rank))
        os.environ.setdefault("WORLD_SIZE", str(world))
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    pkg = importlib.import_module("minion-plasmid-consensus_amd")
    eng = pkg.engine

    cfg = args.config
    n, reads, scaling, profile, seed, antisense, desc = CONFIGS[cfg]
    samples, global_reads = shard_samples(pkg, cfg, rank, world)
    # batches in flight: R independent pipelines (own device copy of the batch,
    # own workspace) on R streams, taken in turn, so one batch's latency-bound
    # post-parse chain overlaps the next batch's parse (a stream of plasmid
    # batches, as a sequencing run produces; every step is still one full pass
    # over one batch)
    R = max(1, args.inflight if args.inflight is not None else INFLIGHT[cfg])
    if world > 1 and args.inflight is None and cfg != "c5":
        # a rank's pipelines each drive a compute stream AND an RCCL communicator
        # stream; a process gets GPU_MAX_HW_QUEUES = 4 hardware queues, and streams
        # beyond that share queues in order (a shared queue can stall one
        # pipeline's collective behind another's compute, on every rank): 2 + 2
        R = min(R, MAX_PIPELINES_DIST)
    # with batches in flight the parse grid is sized for fewer CUs, so the other
    # batch's post-parse kernels (which cannot share a CU with the parse: it holds
    # every VGPR) run beside it; measured per config at its default R
    # (profiles/r03_experiments/parse_cus_inflight.txt, c1_parse_workgroups_inflight.txt);
    # every rank of an N-GPU run does the same (weak scaling: the same per-GPU batch)
    cus = (args.parse_cus if args.parse_cus is not None else PARSE_CUS_INFLIGHT[cfg]) if R > 1 else 0

    # one communicator per pipeline in flight (every rank creates them in the
    # same order): a pipeline's collectives then run on their own RCCL stream
    # instead of queueing behind the other pipeline's on one shared stream
    groups = [dist.new_group(list(range(world))) for _ in range(R)] if use_dist and cfg != "c5" else [None] * R

    def make_runner(parse_cus, group=None):
        if use_dist and cfg != "c5":
            dmod = importlib.import_module("minion-plasmid-consensus_amd.dist")
            return dmod.ShardedPileup([samples], [local], ex=dmod.DistExchange(group), parse_cus=parse_cus)
        return eng.Runner(samples, device=local, parse_cus=parse_cus)

    runners = [make_runner(cus, groups[k]) for k in range(R)]
    streams = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(R - 1)]
    runner = runners[0]

    def step(k):
        with torch.cuda.stream(streams[k % R]):
            runners[k % R].step(mdf, gtf)
    eager_step = step

    def calls_of(r):
        """(max depth, device call rows) of every sample: a step's full result."""
        return [(int(x["max_depth"]), x["raw"].tobytes()) for x in r.fetch()]

    batch = runner.batch
    aligned = batch.aligned_bases
    coll_dev = "cuda" if backend == "nccl" else "cpu"
    if use_dist:
        t = torch.tensor([aligned], dtype=torch.int64, device=coll_dev)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        aligned = int(t.item())

    mdf, gtf = 0.1, 5.0  # config.yaml:38-39 (MIN_BASE_FACTOR, GLOBAL_THRESHOLD_FACTOR)
    for k in range(max(1, args.warmup) * R):
        step(k)
    torch.cuda.synchronize()
    for r in runners:
        r.check()  # data-error flags must be clear (valid synthetic input)

    # distributed path: every pipeline's step -- phase launches, torch glue ops
    # and RCCL collectives -- captured once in a HIP graph and replayed, so a
    # step costs no host dispatch (world size 1 over RCCL, C2: eager 220 us /
    # step with 141 us of host dispatch, replay 202.5 us = the local runner;
    # profiles/r04_experiments/dist_graph_world1.txt).  All ranks capture the
    # same sequence; if any rank fails to, every rank stays eager.  Default at
    # world size > 1 over RCCL (where the eager step's host dispatch and four
    # collectives would otherwise sit on every rank's critical path); parity of
    # the replayed step is pinned by tests/test_dist_gpu.py::test_rccl_world1_*.
    # gloo (host-staged tensors) cannot be captured: always eager.
    graph_note = None
    want_graph = args.graph == "on" or (args.graph == "auto" and world > 1 and backend == "nccl")
    if args.graph == "on" and backend != "nccl":
        graph_note, want_graph = "graph replay needs RCCL (host-staged gloo exchanges): eager steps", False
    if want_graph and use_dist and cfg != "c5":
        graphs, ok = [], 1
        # the eager step's calls (same mdf / gtf): the replayed step must give them
        eager_calls = [calls_of(r) for r in runners]
        try:
            for r in runners:
                g = torch.cuda.CUDAGraph()
                cap = torch.cuda.Stream()
                with torch.cuda.stream(cap):
                    r.step(mdf, gtf)
                    cap.synchronize()
                    with torch.cuda.graph(g, stream=cap):
                        r.step(mdf, gtf)
                graphs.append(g)
            torch.cuda.synchronize()
        except Exception as e:  # noqa: BLE001 (any capture failure: eager)
            ok, graph_note = 0, "capture failed: %s" % str(e)[:200]
        t = torch.tensor([ok], dtype=torch.int64, device=coll_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        if int(t.item()) == 1:
            def step(k):  # noqa: F811 (replaces the eager step)
                with torch.cuda.stream(streams[k % R]):
                    graphs[k % R].replay()
            for k in range(R):
                step(k)
            torch.cuda.synchronize()
            for r in runners:
                r.check()
            # the replayed step's calls equal the eager step's on
            # every pipeline of every rank, else every rank steps eagerly
            same = all(calls_of(r) == c for r, c in zip(runners, eager_calls))
            t = torch.tensor([1 if same else 0], dtype=torch.int64, device=coll_dev)
            dist.all_reduce(t, op=dist.ReduceOp.MIN)
            if int(t.item()) == 1:
                graph_note = "steps replayed from HIP graphs (one per pipeline), calls checked against the eager step"
            else:
                step = eager_step
                graph_note = "a replayed step's calls differed from the eager step's (some rank): eager steps"
        elif graph_note is None:
            graph_note = "another rank failed to capture: eager steps"

    def barrier():
        if use_dist:
            dist.barrier()

    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(k)
    torch.cuda.synchronize()
    barrier()
    dt = time.perf_counter() - t0
    if use_dist:
        t = torch.tensor([dt], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    ms = dt * 1e3 / args.steps
    value = aligned * args.steps / dt

    def kparse_ms(plan, reps, stream, beside=None):
        """Mean K_parse launch (HIP events on its own stream); ``beside``: a step
        of another pipeline enqueued on its stream before each launch."""
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
        for a, b in ev:
            if beside is not None:
                beside()
            a.record(stream)
            plan.profile_kernel(eng.K_PARSE, stream)
            b.record(stream)
        torch.cuda.synchronize()
        return float(np.mean([a.elapsed_time(b) for a, b in ev]))

    # K_parse on the plan that was TIMED: with batches in flight its grid is
    # sized for `cus` CUs and the other batches' steps run beside it
    timed_k_ms = None
    if R > 1:
        def other():  # the other pipelines' steps, as in the timed loop
            for k in range(1, R):
                with torch.cuda.stream(streams[k]):
                    runners[k].step(mdf, gtf)
        timed_k_ms = kparse_ms(runners[0].plan, args.kernel_reps, streams[0], other)
        timed_geo = runners[0].plan.info()
        for k in range(R):
            step(k)  # leave the plans in a clean state
        torch.cuda.synchronize()
        for r in runners:
            r.check()

    # one batch at a time (the latency of a step) and the dominant kernel on a
    # plan whose parse grid spans every CU, like a single batch's
    single_ms = ms
    if cus:
        del runners
        runner = make_runner(0, groups[0])
        runners = [runner]
        for _ in range(max(1, args.warmup)):
            runner.step(mdf, gtf)
        torch.cuda.synchronize()
        runner.check()
        barrier()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(args.steps):
            runner.step(mdf, gtf)
        torch.cuda.synchronize()
        barrier()
        d1 = time.perf_counter() - t1
        if use_dist:
            t = torch.tensor([d1], dtype=torch.float64, device=coll_dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            d1 = float(t.item())
        single_ms = d1 * 1e3 / args.steps
    plan = runner.plan
    stream = torch.cuda.current_stream()
    k_ms = kparse_ms(plan, args.kernel_reps, stream)
    runner.step(mdf, gtf)  # leave the plan in a clean state
    torch.cuda.synchronize()
    for r in runners:
        r.check()
    geo = plan.info()
    alg_bytes = batch.cs_bytes + 24 * batch.n_reads
    achieved = alg_bytes / (k_ms * 1e-3) / 1e9
    traffic, traffic_src = traffic_record(cfg, world)

    cpu = e2e = hbm = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        port = port_baseline(samples, mdf, gtf, cfg)
        ref = reference_record(cfg)
        if ref is not None:
            # the reference script itself (kind "reference"; it cannot run on the GPU
            # box, so it was timed in the build container: profiles/ref_cpu_baseline.json)
            cpu = dict(ref, port=port)
        else:
            cpu = port
    if rank == 0 and world == 1 and args.hbm_config and args.hbm_config != cfg:
        # the same kernel on a workload that does NOT fit the 256 MiB Infinity
        # Cache: C2's 71 MB of input stays L3-resident across launches, C3's 1.2 GB
        # cannot -- the honest HBM fraction
        del runner, runners, plan
        torch.cuda.empty_cache()
        hbm = kernel_roofline(pkg, eng, args.hbm_config, args.kernel_reps, torch)
    if rank == 0 and world == 1 and not args.no_e2e and cfg in E2E_CONFIGS:
        runner = runners = plan = batch = None
        torch.cuda.empty_cache()
        e2e = e2e_cli(pkg, cfg)

    if rank == 0:
        line = {
            "metric": METRIC, "value": value, "unit": "aligned bases/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": ms, "higher_is_better": True,
            "scaling": "strong" if scaling == "strong" else "weak",
            "vs_baseline": None, "dtype": "u8",
            "data": "synthetic: seeded cs-tag generator (SURVEY §8(d) profile), device-resident",
            "config": {"workload": desc, "ref_len": n, "global_reads_per_sample": global_reads,
                       "local_reads": int(len(samples[0]["tstart"])), "samples_per_gpu": len(samples),
                       "profile": profile, "aligned_bases_per_step": aligned,
                       "cs_bytes_gpu0": int(sum(int(s["cs_off"][-1] - s["cs_off"][0]) for s in samples)),
                       "min_depth_factor": mdf, "global_threshold_factor": gtf,
                       "parallelism": ("replicas" if cfg == "c5" else "read-shard") + f"x{world}",
                       "batches_in_flight": R, "parse_cus": cus or 256,
                       "process_group": backend if use_dist else None, "graph": graph_note},
            "single_batch_ms_per_step": single_ms,
            "what": ("value = aligned bases of K steps / wall time with %d batch copies in flight on %d streams "
                     "(pipelined throughput); single_batch_ms_per_step = the same config one batch at a time" % (R, R)
                     if R > 1 else "value = aligned bases of K steps / wall time, one batch at a time"),
            "roofline": {"bound": ROOF_BOUND, "kernel": "K_parse", "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "traffic_record": traffic_src,
                         "alg_bytes_per_launch": alg_bytes, "mean_launch_us": k_ms * 1e3,
                         "plan": "parse grid on all 256 CUs, nothing beside it (a single batch's launch)",
                         "limiter": LIMITER, "input_l3_resident": batch_l3_resident(cfg)},
            "roofline_timed": None if timed_k_ms is None else {
                "bound": ROOF_BOUND, "kernel": "K_parse", "achieved": alg_bytes / (timed_k_ms * 1e-3) / 1e9,
                "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": alg_bytes / (timed_k_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                "mean_launch_us": timed_k_ms * 1e3, "parse_workgroups": timed_geo["parse_workgroups"],
                "plan": "the timed plan: parse grid sized for %d CUs, the other %d batches' steps on their own "
                        "streams beside every launch" % (cus, R - 1)},
            "roofline_hbm": hbm,
            "cpu_baseline": cpu,
            "e2e": e2e,
        }
        line["config"]["parse_geometry"] = geo
        print(json.dumps(line), flush=True)
    if use_dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
