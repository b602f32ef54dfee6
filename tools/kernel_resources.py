#!/usr/bin/env python3
"""Per-kernel register / scratch / occupancy table of one source file's gfx950 compile
(hipcc -Rpass-analysis=kernel-resource-usage): tools/kernel_resources.py csrc/bm_build.hip [-DX=1 ...]."""
import os
import re
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from raytracercuda_amd import build  # noqa: E402

src, extra = sys.argv[1], sys.argv[2:]
with tempfile.TemporaryDirectory() as d:
    cmd = [build.hipcc(), f"--offload-arch={build.ARCH}", "-O3", "-std=c++17", "-fPIC", *build.FP_FLAGS,
           "--offload-device-only", "-c", "-Rpass-analysis=kernel-resource-usage", "-o", os.path.join(d, "x.o"),
           *extra, src]
    out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for ln in out.splitlines():
    m = re.search(r"remark: (?:\s*)(.*?): (.*?) \[-Rpass", ln)
    if not m:
        continue
    k, v = m.group(1).strip(), m.group(2).strip()
    if k == "Function Name":
        name = subprocess.run(["c++filt", v], capture_output=True, text=True).stdout.strip()
        name = name.replace("bm::(anonymous namespace)::", "").split("(")[0]
        cur = {"name": name}
        rows.append(cur)
    elif cur is not None:
        cur[k] = v
cols = ["VGPRs", "AGPRs", "TotalSGPRs", "ScratchSize [bytes/lane]", "SGPRs Spill", "VGPRs Spill",
        "Occupancy [waves/SIMD]", "LDS Size [bytes/block]"]
print(f"{'kernel':60s} " + " ".join(f"{c.split(' ')[0][:10]:>10s}" for c in cols))
for r in rows:
    print(f"{r['name'][:60]:60s} " + " ".join(f"{r.get(c, '-'):>10s}" for c in cols))
