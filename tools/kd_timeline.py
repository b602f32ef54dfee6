#!/usr/bin/env python3
"""Reference-mode march: per-ray work (counting build) and per-wave timeline (diagnostic build).
    python tools/kd_timeline.py [c2|c3|c5|filled]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools import ab_env  # noqa: E402
from raytracercuda_amd import beam, scenes  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "c2"
c = scenes.CONFIGS[name]
ctx = ab_env.Context(device=0, reference_kd=True)
scene = beam.IScene.create(ctx)
keep = beam.upload_meshes(ctx, scene, scenes.scene(c["scene"]))
scene.updateGPUScene(stats=True)
cam = beam.ICamera.create(ctx)
ctx._check(cam.setInitialRays(c["width"], c["height"], *c["rays"]))
rt = beam.IRenderTarget.createOffscreen(ctx, c["width"], c["height"])
n = c["width"] * c["height"]
cnt = cam.traceCounters(c["eye"], scenes.IDENTITY, scene, rt)
print(f"{name}: per ray {cnt[0] / n:.2f} node records, {cnt[1] / n:.2f} face tests, hits {cnt[2]}")
for _ in range(3):
    d = cam.traceProfile(c["eye"], scenes.IDENTITY, scene, rt)
t0, t1 = d[:, 0].astype(np.int64), d[:, 1].astype(np.int64)
base = t0.min()
s, e = (t0 - base) / 100.0, (t1 - base) / 100.0
w3 = d[:, 3].astype(np.uint64)
dur, work = e - s, (w3 & np.uint64(0xFFFFFFFF)).astype(np.int64)
iters = ((w3 >> np.uint64(32)) & np.uint64(0xFFFF)).astype(np.int64)  # the wave's loop iterations
rounds = (w3 >> np.uint64(48)).astype(np.int64)  # its leaf rounds
round_us = d[:, 2].astype(np.float64) / 100.0  # time in its leaf rounds (k_kd_march_coop's diagnostic build)
print(f"waves {d.shape[0]}, span {e.max():.1f} us, last start {s.max():.1f} us")
print(f"wave us: mean {dur.mean():.2f} p50 {np.median(dur):.2f} p90 {np.percentile(dur, 90):.2f} "
      f"p99 {np.percentile(dur, 99):.2f} max {dur.max():.2f}")
print(f"lane-max work per wave: mean {work.mean():.0f} p50 {np.median(work):.0f} p99 {np.percentile(work, 99):.0f} "
      f"max {work.max()}")
for lo, hi in [(0, 1), (1, 50), (50, 200), (200, 1000), (1000, 5000), (5000, 10 ** 9)]:
    m = (work >= lo) & (work < hi)
    if m.any():
        print(f"  work [{lo},{hi}): {m.sum():6d} waves, dur mean {dur[m].mean():8.2f} us max {dur[m].max():8.2f}, "
              f"ns per unit {1e3 * np.mean(dur[m] / np.maximum(work[m], 1)):.1f}")
print("busy waves over time (us: count):",
      [(round(float(t), 0), int(((s <= t) & (e > t)).sum())) for t in np.linspace(0, e.max(), 12)])
order = np.argsort(e)[::-1][:8]
print("last to end (start us, dur us, work, tile x, y):",
      [(round(float(s[i]), 1), round(float(dur[i]), 1), int(work[i]), int(i % ((c["width"] + 7) // 8)),
        int(i // ((c["width"] + 7) // 8))) for i in order])
heavy = np.argsort(dur)[::-1][:12]
print("longest waves (start us, dur us, work, loop iterations, leaf rounds, us in rounds, ns per walk iteration):",
      [(round(float(s[i]), 1), round(float(dur[i]), 1), int(work[i]), int(iters[i]), int(rounds[i]),
        round(float(round_us[i]), 1), round(1e3 * float(dur[i] - round_us[i]) / max(int(iters[i] - rounds[i]), 1)))
       for i in heavy])
m = iters > 0
print(f"waves with work: iterations mean {iters[m].mean():.1f} max {iters.max()}, leaf rounds mean {rounds[m].mean():.1f} "
      f"max {rounds.max()}; ns per iteration (waves > 100 iterations) "
      f"{1e3 * np.median(dur[iters > 100] / iters[iters > 100]) if (iters > 100).any() else 0:.0f}")
