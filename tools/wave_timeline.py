#!/usr/bin/env python3
"""Per-wave timeline of the trace kernel (diagnostic build): when waves start/end, how long the
heavy ones take, and how that relates to their per-lane work."""
import os
import sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools import ab_env  # noqa: E402
from raytracercuda_amd import beam, scenes  # noqa: E402

scene_name = sys.argv[1] if len(sys.argv) > 1 else "bunny"
ctx = ab_env.Context(device=0)
scene = beam.IScene.create(ctx)
keep = beam.upload_meshes(ctx, scene, scenes.scene(scene_name))
scene.updateGPUScene(stats=True)
cam = beam.ICamera.create(ctx)
ctx._check(cam.setInitialRays(1920, 1080, *scenes.RAYS_1080))
rt = beam.IRenderTarget.createOffscreen(ctx, 1920, 1080)
for rep in range(3):
    d = cam.traceProfile(scenes.BUNNY_EYE, scenes.IDENTITY, scene, rt)
t0 = d[:, 0].astype(np.int64); t1 = d[:, 1].astype(np.int64)
base = t0.min()
s = (t0 - base) / 100.0  # us (100 MHz)
e = (t1 - base) / 100.0
dur = e - s
work = d[:, 3].astype(np.int64)
xcc = (d[:, 2] >> 32).astype(np.int64)
print(f"waves {d.shape[0]}, kernel span {e.max():.1f} us, start span {s.max():.1f} us")
print(f"wave duration us: mean {dur.mean():.2f} p50 {np.median(dur):.2f} p99 {np.percentile(dur,99):.2f} max {dur.max():.2f}")
for lo, hi in [(0, 3), (3, 10), (10, 30), (30, 60), (60, 1000)]:
    m = (work >= lo) & (work < hi)
    if m.any():
        print(f"  work [{lo},{hi}): {m.sum():6d} waves, dur mean {dur[m].mean():7.2f} us, max {dur[m].max():7.2f}, us/iter {np.mean(dur[m] / np.maximum(work[m], 1)):.3f}")
top = np.argsort(e)[-10:]
print("last-ending waves: start, end, dur, work, xcc")
for i in top:
    print(f"  {s[i]:8.1f} {e[i]:8.1f} {dur[i]:7.1f} {work[i]:5d} {xcc[i]}")
hist, edges = np.histogram(s, bins=20)
print("start histogram (us):", list(zip(np.round(edges[:-1], 1), hist)))
print("per-XCC end max:", [round(float(e[xcc == k].max()), 1) for k in range(8) if (xcc == k).any()])
