#!/usr/bin/env python3
"""Prototype tokenizer (exp/tok/k_tok.hip) on bench.py workloads: HIP-event
time per launch, and its unit stream against exp/tok/tok_ref.c (CPU).

  python3 exp/tok/run_tok.py [--waves 8192] [--check c1,c2,c4] c2 c3 c4 c5
"""
import argparse
import ctypes
import importlib
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("configs", nargs="+")
    ap.add_argument("--waves", type=int, default=8192)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--check", default="c1,c2,c4")
    ap.add_argument("--lib", default=os.path.join(HERE, "libtok.so"))
    args = ap.parse_args()
    import torch
    pkg = importlib.import_module("minion-plasmid-consensus_amd")
    eng = pkg.engine
    bench = importlib.import_module("bench")
    lib = ctypes.CDLL(os.path.abspath(args.lib))
    lib.tok_launch.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p,
                               ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    ref = ctypes.CDLL(os.path.join(HERE, "libtok_ref.so"))
    ref.tok_ref.restype = ctypes.c_int64
    ref.tok_ref.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64,
                            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64]
    out = {}
    for cfg in args.configs:
        samples, _ = bench.shard_samples(pkg, cfg, 0, 1)
        b = eng.Batch(samples)
        N, B = b.n_reads, b.cs_bytes
        S = max(1024, -(-B // args.waves + 1023) // 1024 * 1024)
        nw = -(-B // S)
        h_off = np.ascontiguousarray(b.h_cs_off, dtype=np.int64)
        rn = np.searchsorted(h_off[:N], np.arange(nw, dtype=np.int64) * S, side="left").astype(np.int64)
        d_rn = torch.from_numpy(rn).cuda()
        units = torch.empty(nw * S, dtype=torch.int32, device="cuda")
        wcount = torch.zeros(nw, dtype=torch.int32, device="cuda")
        st = torch.cuda.current_stream()

        def launch():
            rc = lib.tok_launch(b.t["cs"].data_ptr(), B, b.t["cs_off"].data_ptr(), N, d_rn.data_ptr(), S, nw,
                                units.data_ptr(), wcount.data_ptr(), ctypes.c_void_p(st.cuda_stream))
            assert rc == 0
        for _ in range(3):
            launch()
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * args.reps)]
        for k in range(args.reps):
            ev[2 * k].record(st)
            launch()
            ev[2 * k + 1].record(st)
        torch.cuda.synchronize()
        ts = sorted(ev[2 * k].elapsed_time(ev[2 * k + 1]) * 1e3 for k in range(args.reps))
        us = ts[len(ts) // 2]
        n_units = int(wcount.sum().item())
        alg = B + 4 * n_units + 8 * (N + 1)
        rec = {"lib": os.path.basename(args.lib), "config": cfg, "reads": N, "cs_bytes": B, "waves": nw, "bytes_per_wave": S, "units": n_units,
               "median_us": us, "min_us": ts[0], "max_us": ts[-1], "algorithmic_bytes": alg,
               "GB_per_s": alg / us / 1e3, "units_per_cs_byte": n_units / max(B, 1)}
        if cfg in args.check.split(","):
            t0 = time.time()
            h_cs = b.t["cs"][:B].cpu().numpy()
            r_units = np.zeros(B + 1, dtype=np.uint32)
            r_wc = np.zeros(nw, dtype=np.uint32)
            tot = ref.tok_ref(h_cs.ctypes.data, B, h_off.ctypes.data, N, S, r_units.ctypes.data, r_wc.ctypes.data, nw)
            wc = wcount.cpu().numpy().astype(np.uint32)
            same_counts = bool(np.array_equal(wc, r_wc))
            ok = same_counts and tot == n_units
            if ok:
                cnt = torch.from_numpy(wc.astype(np.int64)).cuda()
                starts = torch.arange(nw, device="cuda", dtype=torch.int64) * S
                offs = torch.cumsum(cnt, 0) - cnt
                idx = torch.repeat_interleave(starts - offs, cnt) + torch.arange(n_units, device="cuda")
                g = units[idx].cpu().numpy().view(np.uint32)
                bad = np.nonzero(g != r_units[:tot])[0]
                ok = len(bad) == 0
                if not ok:
                    k = int(bad[0])
                    rec["first_mismatch"] = {"unit": k, "gpu": hex(int(g[k])), "ref": hex(int(r_units[k])),
                                             "n_bad": int(len(bad))}
            else:
                dw = np.nonzero(wc != r_wc)[0]
                rec["count_mismatch"] = {"ref_total": int(tot), "gpu_total": n_units, "n_waves_bad": int(len(dw)),
                                         "first_wave": int(dw[0]) if len(dw) else -1,
                                         "gpu": int(wc[dw[0]]) if len(dw) else -1,
                                         "ref": int(r_wc[dw[0]]) if len(dw) else -1}
            rec["check"] = "identical" if ok else "MISMATCH"
            rec["check_s"] = round(time.time() - t0, 1)
        print(json.dumps(rec), flush=True)
        out[cfg] = rec
        del units, b
        torch.cuda.empty_cache()
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    with open(os.path.join(REPO, "gpurun_out", "tok_proto.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
