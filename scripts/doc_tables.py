#!/usr/bin/env python3
"""Markdown tables for DESIGN.md / README.md from bench lines (<dir>/<tag>_<cfg>_bench.json).
  python3 scripts/doc_tables.py profiles r03f"""
import json
import os
import sys

d, tag = sys.argv[1], sys.argv[2]
NAMES = {"c1": "C1 5 kb, 20k reads", "c2": "**C2 2.7 kb, 2×100k reads**", "c3": "C3 10 kb, 1 M reads, 1 GPU",
         "c4": "C4 10 kb, 2×100k, indel 1/5/5 %", "c5": "C5 12 × 2 × 10k reads of 30 kb"}
rows, e2e = [], []
for c in ("c1", "c2", "c3", "c4", "c5"):
    p = os.path.join(d, f"{tag}_{c}_bench.json")
    if not os.path.exists(p):
        continue
    b = json.load(open(p))
    rf = b["roofline"]
    g = b["config"]["parse_geometry"]
    tr = rf.get("traffic")
    trs = f"{tr / 1e6:.0f} / {rf['alg_bytes_per_launch'] / 1e6:.0f} MB ({tr / rf['alg_bytes_per_launch']:.1f}×)" if tr else "—"
    cpu = b.get("cpu_baseline") or {}
    ref = cpu.get("value")
    port = (cpu.get("port") or {}).get("value")
    rows.append(f"| {NAMES[c]} | {b['value']:.3g} | {b['ms_per_step'] * 1e3:.0f} | {rf['mean_launch_us']:.0f} | "
                f"{g['tally_mode']}, {g['parse_window'] // 1024} KiB, {g['parse_waves']} | "
                f"{rf['achieved']:.0f} GB/s ({100 * rf['frac']:.1f} %) | {trs} | "
                f"{b['value'] / port:.2g}× | {b['value'] / ref:.2g}× |" if ref and port else "")
    e = b.get("e2e")
    if e:
        ph = e["phases_s"]
        e2e.append(f"| {NAMES[c]} | {e['output_files']} | {e['input_bytes'] / 1e9:.2f} GB | {e['wall_s']:.3f} s | "
                   f"{ph['ingest']:.3f} / {ph['device']:.3f} / {ph['write']:.4f} s | {e['value']:.3g} |")
print("| Config | aligned bases/s | µs/step | K_parse µs | geometry (mode, window, waves) | K_parse achieved (frac of 8 TB/s) | "
      "K_parse HBM traffic / algorithmic | vs C port (1 thread) | vs reference script (1 core) |")
print("|---|---|---|---|---|---|---|---|---|")
print("\n".join(rows))
print()
print("| Config | output files | input files | E2E wall | ingest / device / write | aligned bases/s E2E |")
print("|---|---|---|---|---|---|")
print("\n".join(e2e))
