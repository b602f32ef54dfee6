#!/usr/bin/env python3
"""Summarise one config of a tools/gpu_profile.sh session into profiles/<name>.md + _traffic.json
and copy the raw kernel-stats CSVs next to them.

    python tools/summarize_profile.py gpurun_out/r2_p1 c2 profiles/r02_v1

HBM bytes per launch follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are in KiB; on
gfx950 FETCH_SIZE reads half the bytes of a wide coalesced read, so the read side is reported both as
counted and doubled (the doubled value is the upper estimate bench.py uses as `traffic`); Infinity
Cache hits are counted too, so this is an upper bound on HBM bytes. The limiter block decomposes
wave time (SQ_WAIT_ANY + SQ_WAIT_INST_ANY + SQ_ACTIVE_INST_ANY ~= SQ_WAVE_CYCLES, the guide's PMC
table): a wave parked on s_waitcnt most of its life is bound by the latency of its loads.
The summary carries the box's source stamp: bench.py uses it only for the same source revision.
"""
import collections
import csv
import glob
import json
import os
import shutil
import sys


def short(name):
    n = name.replace("void ", "").replace("bm::(anonymous namespace)::", "")
    n = n.split("(")[0]
    return n[:60]


def kernel_stats(path):
    rows = []
    if os.path.exists(path):
        for r in csv.DictReader(open(path)):
            rows.append((short(r["Name"]), int(r["Calls"]), float(r["AverageNs"]) / 1e3, float(r["MinNs"]) / 1e3,
                         float(r["MaxNs"]) / 1e3, float(r["Percentage"])))
    return rows


def pmc_means(src):
    """counter -> kernel -> mean per dispatch (summing the per-dimension rows of one dispatch)."""
    out = collections.defaultdict(dict)
    for f in sorted(glob.glob(os.path.join(src, "pmc_*", "pmc_counter_collection.csv"))):
        per = collections.defaultdict(float)
        for r in csv.DictReader(open(f)):
            per[(r["Counter_Name"], short(r["Kernel_Name"]), r["Dispatch_Id"])] += float(r["Counter_Value"])
        agg = collections.defaultdict(list)
        for (c, k, _), v in per.items():
            agg[(c, k)].append(v)
        for (c, k), v in agg.items():
            out[c][k] = sum(v) / len(v)
    return out


def limiter(p, k):
    g = lambda c: p.get(c, {}).get(k)  # noqa: E731
    lim = {}
    if g("TCC_HIT_sum") is not None and g("TCC_MISS_sum") is not None and g("TCC_HIT_sum") + g("TCC_MISS_sum") > 0:
        lim["l2_hit"] = g("TCC_HIT_sum") / (g("TCC_HIT_sum") + g("TCC_MISS_sum"))
    if g("TCP_TOTAL_CACHE_ACCESSES_sum") and g("TCP_TCC_READ_REQ_sum") is not None:
        lim["l1_miss_to_l2_per_access"] = g("TCP_TCC_READ_REQ_sum") / g("TCP_TOTAL_CACHE_ACCESSES_sum")
    wc = g("SQ_WAVE_CYCLES")
    if wc:
        for c, name in (("SQ_WAIT_ANY", "wave_time_waiting_on_loads_or_barrier"),
                        ("SQ_WAIT_INST_ANY", "wave_time_issue_stalled"),
                        ("SQ_ACTIVE_INST_ANY", "wave_time_issuing")):
            if g(c) is not None:
                lim[name] = g(c) / wc
    # GRBM_GUI_ACTIVE sums the 8 XCDs' busy cycles (8 x the kernel's cycles); TA/TD are per CU (256)
    if g("TA_TA_BUSY_sum") is not None and g("GRBM_GUI_ACTIVE"):
        lim["ta_busy"] = g("TA_TA_BUSY_sum") / (g("GRBM_GUI_ACTIVE") / 8 * 256)
    if g("TD_TD_BUSY_sum") is not None and g("GRBM_GUI_ACTIVE"):
        lim["td_busy"] = g("TD_TD_BUSY_sum") / (g("GRBM_GUI_ACTIVE") / 8 * 256)
    lim["raw"] = {c: v[k] for c, v in p.items() if k in v}
    w = lim.get("wave_time_waiting_on_loads_or_barrier")
    if w is not None:
        lim["bound_by"] = (f"latency and issue, not HBM: waves parked on s_waitcnt {100 * w:.0f} % of their time, "
                           f"ready but stalled behind other waves' issue "
                           f"{100 * lim.get('wave_time_issue_stalled', float('nan')):.0f} %, issuing "
                           f"{100 * lim.get('wave_time_issuing', float('nan')):.0f} %; L2 hit "
                           f"{100 * lim.get('l2_hit', float('nan')):.1f} %, TA busy "
                           f"{100 * lim.get('ta_busy', float('nan')):.0f} %")
    return lim


def dispatch_durations(trace_csv, prefix):
    """Per-dispatch durations (µs) of the kernels whose short name starts with prefix."""
    if not os.path.exists(trace_csv):
        return []
    return [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in csv.DictReader(open(trace_csv))
            if short(r["Kernel_Name"]).startswith(prefix)]


def median_durations(trace_csv):
    """kernel -> median dispatch duration (µs) of a kernel trace."""
    per = collections.defaultdict(list)
    if os.path.exists(trace_csv):
        for r in csv.DictReader(open(trace_csv)):
            per[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    return {k: sorted(v)[len(v) // 2] for k, v in per.items()}


def main(src_root, cfg, dst_prefix):
    src = os.path.join(src_root, cfg)
    dst = f"{dst_prefix}_{cfg}"
    os.makedirs(os.path.dirname(dst), exist_ok=True)
    stamp = open(os.path.join(src_root, "stamp.txt")).read().strip()
    lines = [f"source stamp `{stamp}` (raytracercuda_amd/build.py:source_stamp of the box's tree)\n"]
    for mode in ("single", "inflight"):
        stats = os.path.join(src, f"prof_{mode}", "bench_kernel_stats.csv")
        rows = kernel_stats(stats)
        if not rows:
            continue
        shutil.copy(stats, f"{dst}_{mode}_kernel_stats.csv")
        lines.append(f"## rocprofv3 --kernel-trace --stats: `bench.py --config {cfg} --only {mode}`\n")
        lines.append("| kernel | calls | avg µs | min µs | max µs | % |")
        lines.append("|---|---|---|---|---|---|")
        for n, c, a, mi, ma, pc in rows:
            lines.append(f"| {n} | {c} | {a:.1f} | {mi:.1f} | {ma:.1f} | {pc:.1f} |")
        d = sorted(dispatch_durations(os.path.join(src, f"prof_{mode}", "bench_kernel_trace.csv"),
                                      "k_trace_quad<false"))
        if d:
            med = d[len(d) // 2]
            lines.append(f"\nk_trace_quad<false...>: {len(d)} dispatches, median {med:.1f} µs "
                         f"(the avg above includes outliers: the run's first dispatch and the untimed reference "
                         f"frame into a fresh target; max {d[-1]:.0f} µs)")
        log = os.path.join(src, f"prof_{mode}.log")
        for ln in open(log) if os.path.exists(log) else []:
            if ln.startswith("{"):
                b = json.loads(ln)
                sf = b.get("single_frame") or {}
                tail = (f", single_frame kernel {sf['trace_kernel_ms']:.4f} ms" if "trace_kernel_ms" in sf
                        else " (frames in flight only)")
                lines.append(f"\nbench line of this run: value {b['value']:.0f} Mrays/s, trace_kernel_ms "
                             f"{b['trace_kernel_ms']:.4f}{tail}\n")
    p = pmc_means(src)
    kern = {}
    names = sorted(set().union(*[set(v) for v in p.values()])) if p else []
    if p:
        lines.append("\n## PMC (separate --pmc passes of `--only single`; mean per dispatch)\n")
        med = median_durations(os.path.join(src, "prof_single", "bench_kernel_trace.csv"))
        # kernels of the in-flight path only: their launch durations there (overlapped with other frames')
        med_if = median_durations(os.path.join(src, "prof_inflight", "bench_kernel_trace.csv"))
        med.update({k: v for k, v in med_if.items() if k not in med})
        lines.append("| kernel | FETCH_SIZE MB (counted) | read MB (x2 gfx950) | WRITE_SIZE MB | L2 hit | wave time on "
                     "s_waitcnt | median µs | HBM GB/s (read x2 + write) | of 8 TB/s |")
        lines.append("|---|---|---|---|---|---|---|---|---|")
        for k in names:
            f = p.get("FETCH_SIZE", {}).get(k)
            w = p.get("WRITE_SIZE", {}).get(k)
            lim = limiter(p, k)
            kern[k] = {"read_bytes_counted": f * 1024 if f is not None else None,
                       "read_bytes_x2": 2 * f * 1024 if f is not None else None,
                       "write_bytes": w * 1024 if w is not None else None, "limiter": lim}
            fs = f"{f * 1024 / 1e6:.2f}" if f is not None else "-"
            f2 = f"{2 * f * 1024 / 1e6:.2f}" if f is not None else "-"
            ws = f"{w * 1024 / 1e6:.2f}" if w is not None else "-"
            l2 = f"{100 * lim['l2_hit']:.1f} %" if "l2_hit" in lim else "-"
            wt = lim.get("wave_time_waiting_on_loads_or_barrier")
            us = med.get(k)
            hbm = (2 * f + w) * 1024 if f is not None and w is not None else None
            gbs = hbm / (us * 1e3) if hbm is not None and us else None
            lines.append(f"| {k} | {fs} | {f2} | {ws} | {l2} | {'-' if wt is None else f'{100 * wt:.0f} %'} | "
                         f"{'-' if us is None else f'{us:.1f}'} | {'-' if gbs is None else f'{gbs:.0f}'} | "
                         f"{'-' if gbs is None else f'{gbs / 8000:.3f}'} |")
        lines.append("\nmedian µs: dispatch durations of the `--only single` kernel trace; k_cull and k_trace_rays run only "
                     "in flight, so theirs are in-flight launch durations (overlapped with the other frames' launches, "
                     "so their GB/s understate what one launch alone reaches). Counter bytes include Infinity Cache "
                     "hits (an upper bound on HBM bytes).")
        lines.append("\nRaw counters per kernel: see the `_traffic.json` next to this file.")
    with open(dst + "_traffic.json", "w") as fj:
        json.dump({"source": src, "config": cfg, "stamp": stamp,
                   "note": "rocprofv3 --pmc, separate passes, mean per dispatch of bench.py --only single; "
                           "FETCH_SIZE x2 per MI355X_MICROARCH.md (gfx950)", "kernels": kern}, fj, indent=1)
    with open(dst + ".md", "w") as f:
        f.write(f"# Profile {os.path.basename(dst)} (from {src})\n\n" + "\n".join(lines) + "\n")
    print(dst + ".md")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3])
