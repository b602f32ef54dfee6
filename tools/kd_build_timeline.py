#!/usr/bin/env python3
"""Reference-mode kd build timeline from a rocprofv3 kernel trace of tools/kd_build_bench.py: each build
(from its k_gather to the next build's) as kernel start offsets, durations and the gaps between them,
for the last builds of the trace (steady state).
    python tools/kd_build_timeline.py gpurun_out/TAG/kd/pmc_kernel_trace.csv [builds]"""
import csv
import sys


def main(path, nshow=2):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    builds, cur = [], None
    for r in rows:
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("bm::", "").replace("void ", "")
        name = name.split("(")[0]
        if name.startswith("k_gather"):
            cur = []
            builds.append(cur)
        if cur is not None:
            cur.append((name, int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    spans = []
    for b in builds:
        # the build ends at its last kernel before the next k_gather; marches of other tools are not traced here
        spans.append((b[-1][2] - b[0][1]) / 1000.0)
    print(f"{len(builds)} builds; spans (first kernel start -> last kernel end) us: "
          + " ".join(f"{s:.1f}" for s in spans))
    for b in builds[-nshow:]:
        t0 = b[0][1]
        prev_end = t0
        busy = 0.0
        print(f"-- build: span {(b[-1][2] - t0) / 1000:.1f} us")
        for name, s, e in b:
            gap = (s - prev_end) / 1000.0
            busy += (e - s) / 1000.0
            print(f"  {(s - t0) / 1000:8.1f} +{(e - s) / 1000:7.1f}  gap {gap:6.1f}  {name[:70]}")
            prev_end = max(prev_end, e)
        print(f"  kernels {busy:.1f} us of {(b[-1][2] - t0) / 1000:.1f}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 2)
