#!/usr/bin/env python3
"""One rank's work of an N-GPU bench run, on ONE GPU.

  python3 scripts/shard_probe.py --config c3 --world 8 --mode parse [--reps 5]
      rank 0's shard of the N-shard plan (bench.shard_samples(cfg, 0, N): C3 the
      first 1M/N reads, C1/C2/C4 the first per-GPU slice of an N x larger global
      read set), parse grid on all CUs as in bench.py's roofline plan; runs
      the parse phase (K_clear + K_parse [+ K_subs]) --reps times.  Under
      rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE this is the per-rank K_parse
      traffic bench.py reports on an N-GPU line (scripts/shard_traffic.sh ->
      profiles/pmc_traffic_<cfg>_w<N>.json).
  python3 scripts/shard_probe.py --config c3 --world 8 --mode step [--reps 5]
      all N shards in this process (dist.ShardedPileup, LocalExchange: torch
      ops stand in for the four collectives), --reps steps.  Under rocprofv3
      --kernel-trace --stats every pipeline kernel runs N times per step on a
      shard of one rank's size: the per-rank step of the N-GPU run without its
      collectives (scripts/shard_step.sh -> profiles/r06_shards/).
"""
import argparse
import importlib
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--mode", choices=("parse", "step"), default="parse")
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    import torch
    bench = importlib.import_module("bench")
    pkg = importlib.import_module("minion-plasmid-consensus_amd")
    eng = pkg.engine
    dist = importlib.import_module("minion-plasmid-consensus_amd.dist")
    cfg, W = args.config, args.world
    mdf, gtf = 0.1, 5.0
    t0 = time.time()
    if args.mode == "parse":
        samples, total = bench.shard_samples(pkg, cfg, 0, W)
        strands = len(samples)
        n_local = sum(len(s["tstart"]) for s in samples)
        batch = eng.Batch(samples, read_offset=0, n_reads_global=total * strands, shard=0, n_shards=W)
        plan = eng.Plan(batch)
        for _ in range(args.reps):
            plan.phase("parse")
        torch.cuda.synchronize()
        st = plan.status()
        assert int(st[eng.MPC_ST_FLAGS]) == 0, st
        rec = {"config": cfg, "world": W, "mode": "parse", "local_reads": n_local, "global_reads": total * strands,
               "cs_bytes": batch.cs_bytes, "alg_bytes_per_launch": batch.cs_bytes + 24 * batch.n_reads,
               "aligned_bases": batch.aligned_bases, "geometry": plan.info()}
    else:
        # the whole global read set of an N-GPU run (strong: the config's reads;
        # weak: N x the per-GPU reads), split into N contiguous shards
        n, reads, scaling, profile, seed, anti, _ = bench.CONFIGS[cfg]
        syn = pkg.synth.Synth(n=n, n_reads=reads * (W if scaling == "weak" else 1), profile=profile, seed=seed,
                              antisense=anti)
        samples = [syn.sample(s) for s in range(2 if anti else 1)]
        sp = dist.ShardedPileup(dist.split_samples(samples, W), [0] * W)
        sp.step(mdf, gtf)
        torch.cuda.synchronize()
        sp.check()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.reps)]
        for a, b in ev:
            a.record()
            sp.step(mdf, gtf)
            b.record()
        torch.cuda.synchronize()
        sp.check()
        ms = sorted(a.elapsed_time(b) for a, b in ev)
        rec = {"config": cfg, "world": W, "mode": "step", "shard_reads": [b.n_reads for b in sp.batches],
               "all_shards_step_ms_median": ms[len(ms) // 2],
               "note": "all N shards of one step, sequentially on one GPU, LocalExchange torch ops in place of "
                       "the collectives; per-rank kernels = rocprofv3 stats / N"}
    rec["wall_s"] = time.time() - t0
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
