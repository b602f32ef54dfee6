#!/usr/bin/env python3
"""Mean per-dispatch PMC values of the trace kernels in a pmc_compare.sh output dir."""
import collections
import csv
import glob
import os
import sys

src = sys.argv[1]
rows = collections.defaultdict(list)
for f in sorted(glob.glob(os.path.join(src, "*", "pmc_counter_collection.csv"))):
    var = os.path.basename(os.path.dirname(f)).split("_")[0]
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "k_trace" not in k and "k_cull" not in k:
            continue
        name = k.replace("void bm::(anonymous namespace)::", "").split("(")[0]
        # PMC values are per dispatch and per counter; several dimensions sum into one row already
        rows[(var, name, r["Counter_Name"])].append((int(r["Dispatch_Id"]), float(r["Counter_Value"])))
out = collections.defaultdict(dict)
for (var, name, ctr), vals in rows.items():
    per = collections.defaultdict(float)
    for d, v in vals:
        per[d] += v
    out[(var, name)][ctr] = sum(per.values()) / len(per)
for (var, name), d in sorted(out.items()):
    print(f"{var} {name}")
    for k in sorted(d):
        print(f"    {k:34s} {d[k]:16.1f}")
