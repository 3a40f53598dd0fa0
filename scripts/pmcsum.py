#!/usr/bin/env python3
"""Per-kernel mean of rocprofv3 --pmc counters: python3 scripts/pmcsum.py <dir> [kernel-substring...]"""
import csv, glob, sys, collections
d = sys.argv[1]
pats = sys.argv[2:] or ["K_"]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "")
        if not any(p in name for p in pats):
            continue
        key = name.split("(")[0]
        acc[key][(r["Dispatch_Id"], r["Counter_Name"])].append(float(r["Counter_Value"]))
for k, v in sorted(acc.items()):
    per = collections.defaultdict(list)
    for (disp, cn), vals in v.items():
        per[cn].append(sum(vals))
    print(k)
    for cn in sorted(per):
        xs = per[cn]
        print("   %-24s %16.1f  (n=%d)" % (cn, sum(xs) / len(xs), len(xs)))
