#!/usr/bin/env python3
"""Median per-kernel duration of the build (and refit) launches in rocprofv3 kernel traces of
tools/build_bench.py, one trace per scene: tools/build_kernels.py gpurun_out/<tag>."""
import collections
import csv
import glob
import os
import statistics
import sys


def short(n):
    return n.replace("void ", "").replace("bm::(anonymous namespace)::", "").split("(")[0]


for d in sorted(glob.glob(os.path.join(sys.argv[1], "k_*"))):
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if not f:
        continue
    rows = sorted(csv.DictReader(open(f[0])), key=lambda r: int(r["Start_Timestamp"]))
    per = collections.defaultdict(list)
    builds = []
    cur = None
    for r in rows:
        k = short(r["Kernel_Name"])
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        if k.startswith("k_gather"):
            cur = [int(r["Start_Timestamp"]), int(r["End_Timestamp"]), []]
            builds.append(cur)
        if cur is not None and k.startswith("k_"):
            cur[1] = int(r["End_Timestamp"])
            cur[2].append((k, dur))
    full = [b for b in builds if any(k.startswith("k_morton") for k, _ in b[2])][2:]
    print(f"== {os.path.basename(d)[2:]}: {len(full)} builds, span median "
          f"{statistics.median((b[1] - b[0]) / 1e3 for b in full):.1f} us")
    ks = collections.defaultdict(list)
    for b in full:
        seen = collections.Counter()
        for k, dur in b[2]:
            seen[k] += 1
            ks[f"{k}#{seen[k]}" if seen[k] > 1 or k.startswith("k_onesweep") else k].append(dur)
    for k, v in ks.items():
        print(f"   {k:40s} {statistics.median(v):7.1f} us")
