#!/usr/bin/env python3
"""Summarise a gpu_session.sh output dir (rocprofv3 kernel stats + PMC passes + bench line) into
profiles/<name>.md and copy the raw kernel-stats CSV next to it.

    python tools/summarize_profile.py gpurun_out/r1c profiles/r01_bunny1080

HBM bytes per launch follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are in KiB;
on gfx950 FETCH_SIZE reads half the bytes of a wide coalesced read, so the read side is reported
both as counted and doubled (the doubled value is the upper estimate used as `traffic`).
"""
import collections
import csv
import json
import os
import shutil
import sys


def short(name):
    n = name.replace("void ", "").replace("bm::(anonymous namespace)::", "")
    n = n.split("(")[0]
    return n[:60]


def main(src, dst):
    os.makedirs(os.path.dirname(dst), exist_ok=True)
    stats = os.path.join(src, "prof", "bench_kernel_stats.csv")
    lines = []
    if os.path.exists(stats):
        shutil.copy(stats, dst + "_kernel_stats.csv")
        lines.append("## rocprofv3 --kernel-trace --stats (bench.py, same command)\n")
        lines.append("| kernel | calls | avg µs | min µs | max µs | % |")
        lines.append("|---|---|---|---|---|---|")
        for r in csv.DictReader(open(stats)):
            lines.append(f"| {short(r['Name'])} | {r['Calls']} | {float(r['AverageNs']) / 1e3:.1f} | "
                         f"{float(r['MinNs']) / 1e3:.1f} | {float(r['MaxNs']) / 1e3:.1f} | {float(r['Percentage']):.1f} |")
    pmc = {}
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        p = os.path.join(src, f"pmc_{ctr}", "pmc_counter_collection.csv")
        if not os.path.exists(p):
            continue
        agg = collections.defaultdict(list)
        for r in csv.DictReader(open(p)):
            agg[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
        pmc[ctr] = {k: sum(v) / len(v) for k, v in agg.items()}
    if pmc:
        lines.append("\n## PMC: HBM traffic per launch (separate --pmc passes, KiB -> MB)\n")
        lines.append("| kernel | FETCH_SIZE MB (counted) | read MB (x2 gfx950 correction) | WRITE_SIZE MB |")
        lines.append("|---|---|---|---|")
        names = sorted(set().union(*[set(v) for v in pmc.values()]))
        for k in names:
            f = pmc.get("FETCH_SIZE", {}).get(k)
            w = pmc.get("WRITE_SIZE", {}).get(k)
            fs = f"{f * 1024 / 1e6:.2f}" if f is not None else "-"
            f2 = f"{2 * f * 1024 / 1e6:.2f}" if f is not None else "-"
            ws = f"{w * 1024 / 1e6:.2f}" if w is not None else "-"
            lines.append(f"| {k} | {fs} | {f2} | {ws} |")
        # machine-readable per-launch bytes for bench.py's roofline.traffic
        kern = {}
        for k in names:
            f = pmc.get("FETCH_SIZE", {}).get(k)
            w = pmc.get("WRITE_SIZE", {}).get(k)
            kern[k] = {"read_bytes_counted": f * 1024 if f is not None else None,
                       "read_bytes_x2": 2 * f * 1024 if f is not None else None,
                       "write_bytes": w * 1024 if w is not None else None}
        with open(dst + "_traffic.json", "w") as fj:
            json.dump({"source": src, "note": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes, "
                       "mean per launch; FETCH_SIZE x2 per MI355X_MICROARCH.md (gfx950)", "kernels": kern},
                      fj, indent=1)
    bench = os.path.join(src, "bench.log")
    if os.path.exists(bench):
        for ln in open(bench):
            if ln.startswith("{"):
                lines.append("\n## bench.py line\n")
                lines.append("```json\n" + json.dumps(json.loads(ln), indent=1) + "\n```")
    with open(dst + ".md", "w") as f:
        f.write(f"# Profile {os.path.basename(dst)} (from {src})\n\n" + "\n".join(lines) + "\n")
    print(dst + ".md")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
