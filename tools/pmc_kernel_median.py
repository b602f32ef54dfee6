#!/usr/bin/env python3
"""Median per-dispatch counter value (MB for *_SIZE) of the trace kernels in rocprofv3 --pmc outputs:
    python tools/pmc_kernel_median.py gpurun_out/TAG/pmc_*_SIZE"""
import collections
import csv
import statistics
import sys

for d in sys.argv[1:]:
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(d + "/pmc_counter_collection.csv")):
        n = r["Kernel_Name"].replace("void ", "").replace("bm::(anonymous namespace)::", "").replace("bm::", "")
        if n.startswith(("k_trace", "k_cull")):
            scale = 1024 / 1e6 if r["Counter_Name"].endswith("_SIZE") else 1.0
            agg[n.split("(")[0]].append(float(r["Counter_Value"]) * scale)
    for k, v in sorted(agg.items()):
        print(f"{d.rstrip('/').split('/')[-1]:36s} {k:42s} n={len(v):3d} median {statistics.median(v):8.2f}")
