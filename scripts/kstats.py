#!/usr/bin/env python3
"""Print a rocprofv3 kernel_stats.csv compactly: python3 scripts/kstats.py <dir>"""
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
for r in rows[: int(sys.argv[2]) if len(sys.argv) > 2 else 20]:
    name = r["Name"].replace("(anonymous namespace)::", "")[:58]
    print("%-58s %6s %11.1f us avg %6s%%" % (name, r["Calls"], float(r["AverageNs"]) / 1e3, r["Percentage"][:5]))
