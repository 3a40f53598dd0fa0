#!/usr/bin/env python3
"""Benchmark: aligned bases/s of pileup + consensus on MI355X (BASELINE.json metric).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2]

A step = one full pass of the hot path (Steps 4-6 of the reference:
cs parse -> pileup -> consensus calls) over one batch of synthetic, seeded,
device-resident input.  At N=1 the workload is BASELINE.json configs[1]
(C2: pUC19-size 2,686 bp plasmid, 100k reads, sense + antisense in one launch).
With N>1 (torch.distributed.run, one rank per GPU, RCCL) every rank holds a
C2-sized contiguous read shard of ONE global pileup (weak scaling) and the
ranks exchange the downstream-event index and the count rows (see
minion-plasmid-consensus_amd/dist.py).

Output: one JSON line (rank 0) with the contract fields plus
  roofline      the dominant kernel (K_parse) vs the HBM roofline: algorithmic
                bytes (sum of cs bytes + 24 B per read) / its mean
                duration measured here with HIP events on the launch stream
  cpu_baseline  the C restatement of the reference (oracle/, "port") timed on
                this host on the full C2 workload, 1 thread (rank 0, N=1 only)
"""
import argparse
import importlib
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "aligned bases/sec pileup+consensus (1/2/4/8 GPU) and % HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)

CONFIGS = {
    # name: (n, reads per sample per rank, profile, seed, antisense, description)
    "c2": (2686, 100_000, "default", 2, True,
           "C2 (BASELINE configs[1]): pUC19-size 2,686 bp plasmid, 100k reads, sense+antisense pileup"),
    "c1": (5000, 20_000, "default", 1, False,
           "C1 (BASELINE configs[0]): 5 kb plasmid, 20k reads, sense only"),
    "c3": (10_000, 125_000, "default", 3, False,
           "C3 (BASELINE configs[2]): 10 kb plasmid, 1M reads total over 8 GPUs (125k per GPU), sense"),
    "c4": (10_000, 100_000, "indel", 4, True,
           "C4 (BASELINE configs[3]): 10 kb, 100k reads, indel-heavy 1/5/5 %, sense+antisense"),
    # multi-sample: 96 plasmids partitioned over the ranks (12 per GPU at N=8), both strands,
    # replicas only (no collective); at N=1 one GPU holds the 12 plasmids of rank 0
    "c5": (30_000, 10_000, "default", 5000, True,
           "C5 (BASELINE configs[4]): 30 kb BAC-size constructs, 12 plasmids x 10k reads per GPU "
           "(96 over 8 GPUs), sense+antisense, sample-partitioned"),
}
C5_PER_GPU = 12


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--kernel-reps", type=int, default=20)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--traffic-file", default=os.path.join(REPO, "profiles", "pmc_traffic.json"),
                    help="per-launch HBM bytes of K_parse measured with rocprofv3 --pmc (see profiles/)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one rank per GPU; the modulo only matters for rehearsals with more ranks than GPUs
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    # RCCL ("nccl") over xGMI; MPC_DIST_BACKEND=gloo rehearses the N>1 path on one GPU
    backend = os.environ.get("MPC_DIST_BACKEND", "nccl")
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    pkg = importlib.import_module("minion-plasmid-consensus_amd")
    eng = pkg.engine

    n, reads, profile, seed, antisense, desc = CONFIGS[args.config]
    if args.config == "c5":  # this rank's plasmids (distinct references), both strands
        samples = []
        for k in range(C5_PER_GPU):
            syn = pkg.synth.Synth(n=n, n_reads=reads, profile=profile, seed=seed + C5_PER_GPU * rank + k,
                                  antisense=antisense)
            samples += [syn.sample(s) for s in range(2 if antisense else 1)]
    else:  # every rank generates its own contiguous shard of the global read list
        syn = pkg.synth.Synth(n=n, n_reads=reads, profile=profile, seed=seed + 7919 * rank, antisense=antisense)
        samples = [syn.sample(s) for s in range(2 if antisense else 1)]
    if world > 1 and args.config != "c5":
        dmod = importlib.import_module("minion-plasmid-consensus_amd.dist")
        runner = dmod.ShardedPileup([samples], [local], ex=dmod.DistExchange())
    else:
        runner = eng.Runner(samples, device=local)
    batch = runner.batch
    aligned = batch.aligned_bases  # weak scaling: every rank holds a C2-sized shard of one pileup
    coll_dev = "cuda" if backend == "nccl" else "cpu"
    if world > 1:
        t = torch.tensor([aligned], dtype=torch.int64, device=coll_dev)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        aligned = int(t.item())

    mdf, gtf = 0.1, 5.0  # config.yaml:38-39 (MIN_BASE_FACTOR, GLOBAL_THRESHOLD_FACTOR)
    for _ in range(max(1, args.warmup)):
        runner.step(mdf, gtf)
    runner.check()  # data-error flags must be clear (valid synthetic input)
    torch.cuda.synchronize()

    def barrier():
        if world > 1:
            dist.barrier()

    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        runner.step(mdf, gtf)
    torch.cuda.synchronize()
    barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    ms = dt * 1e3 / args.steps
    value = aligned * args.steps / dt

    # dominant kernel: K_parse, timed live with HIP events on the launch stream
    plan = runner.plan
    stream = torch.cuda.current_stream()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.kernel_reps)]
    for a, b in ev:
        a.record(stream)
        plan.profile_kernel(eng.K_PARSE)
        b.record(stream)
    torch.cuda.synchronize()
    k_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    runner.step(mdf, gtf)  # leave the plan in a clean state
    torch.cuda.synchronize()
    alg_bytes = batch.cs_bytes + 24 * batch.n_reads
    achieved = alg_bytes / (k_ms * 1e-3) / 1e9
    traffic = None
    try:
        tr = json.load(open(args.traffic_file))
        if tr.get("config") == args.config and tr.get("kernel") == "K_parse":
            traffic = tr.get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        pass

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(REPO, "oracle"))
        import oracle  # CPU checker: timed here as the baseline, never on the product path
        c0 = time.perf_counter()
        cb = 0
        for s in samples:
            oracle.run_packed(s["ref"], s["cs"], s["cs_off"], s["tstart"], s["up"], s["up_off"], s["down"],
                              s["down_off"], mdf, gtf)
            cb += int(s["aligned"].sum())
        cdt = time.perf_counter() - c0
        cpu = {"value": cb / cdt, "unit": "aligned bases/s", "cores": 1, "kind": "port",
               "sample": f"full {args.config} workload ({len(samples)} samples x {reads} reads, {cb} aligned bases) "
                         f"through oracle/mpc_oracle.c, 1 thread, {cdt:.2f} s"}

    if rank == 0:
        line = {
            "metric": METRIC, "value": value, "unit": "aligned bases/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": ms, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "u8",
            "data": "synthetic: seeded cs-tag generator (SURVEY §8(d) profile), device-resident",
            "config": {"workload": desc, "ref_len": n, "reads_per_sample_per_gpu": reads,
                       "samples": len(samples), "profile": profile, "aligned_bases_per_step": aligned,
                       "cs_bytes_per_gpu": batch.cs_bytes, "min_depth_factor": mdf,
                       "global_threshold_factor": gtf},
            "roofline": {"bound": "hbm", "kernel": "K_parse", "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "alg_bytes_per_launch": alg_bytes, "mean_launch_us": k_ms * 1e3},
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
