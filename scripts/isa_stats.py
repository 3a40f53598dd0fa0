#!/usr/bin/env python3
"""Register / spill / scratch summary of the K_parse instantiations in a
device-only assembly file (hipcc --cuda-device-only -S).
  python3 scripts/isa_stats.py file.s [kernel-substring]"""
import re
import sys

s = open(sys.argv[1]).read()
want = sys.argv[2] if len(sys.argv) > 2 else "K_parse"
meta = s[s.find("amdhsa.kernels:"):]
for blk in re.split(r"\n  - ", meta)[1:]:
    nm, vg = re.search(r"\.name:\s+(\S+)", blk), re.search(r"\.vgpr_count:\s+(\d+)", blk)
    if not nm or not vg:
        continue
    name = nm.group(1)
    if want not in name:
        continue
    g = lambda k: (re.search(r"\." + k + r":\s+(\d+)", blk) or [None, "?"])[1]
    print("%-60s vgpr %3s sgpr %3s vspill %3s sspill %3s scratch %5s lds %6s" % (
        name[:60], vg.group(1), g("sgpr_count"), g("vgpr_spill_count"), g("sgpr_spill_count"),
        g("private_segment_fixed_size"), g("group_segment_fixed_size")))
