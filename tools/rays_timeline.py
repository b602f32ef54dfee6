#!/usr/bin/env python3
"""Per-wave timeline of k_trace_rays (the in-flight path's trace kernel; diagnostic build via
bm_camera_trace_profile on a render target with its own stream): how the kernel's span splits into
the bulk and the tail, and which waves make the tail.
    python tools/rays_timeline.py [c2|c3|c5] ..."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from tools import ab_env  # noqa: E402
from raytracercuda_amd import beam, scenes  # noqa: E402

for name in sys.argv[1:] or ["c3"]:
    c = scenes.CONFIGS[name]
    ctx = ab_env.Context(device=0)
    ctx.set_param("trace_variant", 12)  # TRACE_COMPACT: k_cull + k_trace_rays, as frames in flight run
    sc = beam.IScene.create(ctx)
    keep = beam.upload_meshes(ctx, sc, scenes.scene(c["scene"]))
    sc.updateGPUScene(stats=True)
    cam = beam.ICamera.create(ctx)
    ctx._check(cam.setInitialRays(c["width"], c["height"], *c["rays"]))
    rt = beam.IRenderTarget.createOffscreen(ctx, c["width"], c["height"])
    s = torch.cuda.Stream()
    rt.setStream(s.cuda_stream)
    for _ in range(3):
        d = cam.traceProfile(c["eye"], scenes.IDENTITY, sc, rt)
    print(f"{name}: trace kind {rt.traceKind()}")
    t0 = d[:, 0].astype(np.int64)
    t1 = d[:, 1].astype(np.int64)
    base = t0.min()
    st, en = (t0 - base) / 100.0, (t1 - base) / 100.0
    dur, work = en - st, d[:, 3].astype(np.int64)
    span = en.max()
    print(f"  waves {d.shape[0]}, span {span:.1f} us, last start {st.max():.1f} us")
    print(f"  wave duration us: p50 {np.median(dur):.1f} p90 {np.percentile(dur, 90):.1f} "
          f"p99 {np.percentile(dur, 99):.1f} max {dur.max():.1f}")
    for f in (0.5, 0.9, 0.99):
        print(f"  {int(f * 100)} % of waves done by {np.percentile(en, f * 100):.1f} us")
    busy = [(np.sum((st <= t) & (en > t))) for t in np.linspace(0, span, 11)]
    print("  waves running at 0, 10, ..., 100 % of the span:", busy)
    top = np.argsort(en)[-8:]
    print("  last-ending waves: start end dur work")
    for i in top:
        print(f"    {st[i]:7.1f} {en[i]:7.1f} {dur[i]:7.1f} {work[i]:6d}")
    w = work.astype(np.float64)
    print(f"  work per wave: p50 {np.median(w):.0f} p99 {np.percentile(w, 99):.0f} max {w.max():.0f}; "
          f"us per work unit (heavy waves) {np.median(dur[w > np.percentile(w, 90)] / w[w > np.percentile(w, 90)]):.3f}")
