"""Calibrate the L1 -> L2 request size on gfx950 (tools/pmc.py L2_READ_REQ_BYTES, L2_WRITE_REQ_BYTES): run tools/micro/l2_calib under
rocprofv3 --pmc with the L2-request counters and divide each kernel's known byte count by its requests.
Measurement infrastructure (GPU box):  python tools/l2_calib.py OUTDIR"""
import os
import statistics
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from tools import pmc  # noqa: E402

MIB64 = 64 << 20
KNOWN = {"k_read16": ("read", MIB64), "k_read4": ("read", MIB64), "k_rec112": ("read", (1 << 19) * 112),
         "k_write16": ("write", MIB64), "k_write4": ("write", MIB64)}
COUNTERS = ("TCP_TCC_READ_REQ_sum", "TCP_TCC_WRITE_REQ_sum", "TCP_TOTAL_CACHE_ACCESSES_sum", "TCC_REQ_sum")


def main():
    out = os.path.abspath(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/l2_calib")
    os.makedirs(out, exist_ok=True)
    exe = os.path.join(REPO, "tools", "micro", "l2_calib")
    cmd = ["timeout", "-s", "KILL", "60", "rocprofv3", "--pmc", *COUNTERS, "--kernel-trace", "--output-format", "csv",
           "-d", out, "-o", "calib", "--", exe]
    rc = subprocess.run(cmd, cwd="/tmp", env=dict(os.environ, TMPDIR="/tmp")).returncode
    if rc:
        sys.exit(rc)
    per = {}
    for d in pmc.read_dispatches(out):
        per.setdefault(d[1], []).append(d[2])
    lines = ["| kernel | bytes | TCP_TCC_READ_REQ | TCP_TCC_WRITE_REQ | TCP tag accesses | TCC_REQ | bytes per request |",
             "|---|---|---|---|---|---|---|"]
    for k, (kind, nbytes) in KNOWN.items():
        runs = per.get(k, [])[1:]  # the first repetition warms up
        if not runs:
            continue
        med = {c: statistics.median(r.get(c, 0.0) for r in runs) for c in COUNTERS}
        req = med["TCP_TCC_READ_REQ_sum" if kind == "read" else "TCP_TCC_WRITE_REQ_sum"]
        lines.append(f"| {k} | {nbytes} | {med['TCP_TCC_READ_REQ_sum']:.0f} | {med['TCP_TCC_WRITE_REQ_sum']:.0f} | "
                     f"{med['TCP_TOTAL_CACHE_ACCESSES_sum']:.0f} | {med['TCC_REQ_sum']:.0f} | "
                     f"{nbytes / req if req else float('nan'):.1f} |")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
