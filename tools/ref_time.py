#!/usr/bin/env python3
"""Reference-mode (kd-tree) trace time on a config's frame, HIP events over 20 traces.
    python tools/ref_time.py [c2|c3|c5|filled] ...   (BM_KD_VARIANT selects the march variant)"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import time  # noqa: E402

import numpy as np  # noqa: E402
import torch  # noqa: E402

from tools import ab_env  # noqa: E402
from raytracercuda_amd import beam, scenes  # noqa: E402

st = torch.cuda.current_stream()
for name in sys.argv[1:] or ["c2"]:
    c = scenes.CONFIGS[name]
    ctx = ab_env.Context(device=0, stream=st.cuda_stream, reference_kd=True)
    sc = beam.IScene.create(ctx)
    keep = beam.upload_meshes(ctx, sc, scenes.scene(c["scene"]))
    b = [sc.updateGPUScene(stats=True)["build_ms"] for _ in range(3)]
    cam = beam.ICamera.create(ctx)
    cam.setInitialRays(c["width"], c["height"], *c["rays"])
    rt = beam.IRenderTarget.createOffscreen(ctx, c["width"], c["height"])
    for _ in range(3):
        ctx._check(cam.trace(c["eye"], scenes.IDENTITY, sc, rt))
    a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(st)
    for _ in range(20):
        ctx._check(cam.trace(c["eye"], scenes.IDENTITY, sc, rt))
    e.record(st)
    torch.cuda.synchronize()
    ms = a.elapsed_time(e) / 20
    ref = rt.read()
    hits = int((ref["tri_id"] != 0xFFFFFFFF).sum())
    print(f"{name} variant {os.environ.get('BM_KD_VARIANT', '2')}: build {b[-1]:.3f} ms, trace {ms:.3f} ms = "
          f"{c['width'] * c['height'] / ms / 1e6:.2f} Grays/s, hits {hits}", flush=True)
    # frames in flight: NBUF render targets, each on its own HIP stream (as bench.py's value)
    for nbuf in (2, 3):
        rts = [beam.IRenderTarget.createOffscreen(ctx, c["width"], c["height"]) for _ in range(nbuf)]
        streams = [torch.cuda.Stream() for _ in range(nbuf)]
        for r, s_ in zip(rts, streams):
            r.setStream(s_.cuda_stream)
        for i in range(6):
            ctx._check(cam.trace(c["eye"], scenes.IDENTITY, sc, rts[i % nbuf]))
        ctx.sync()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(60):
            ctx._check(cam.trace(c["eye"], scenes.IDENTITY, sc, rts[i % nbuf]))
        ctx.sync()
        torch.cuda.synchronize()
        per = (time.perf_counter() - t0) / 60 * 1e3
        same = all(np.array_equal(rts[0].read()[k], ref[k]) for k in ref)
        print(f"   {nbuf} frames in flight: {per:.3f} ms per frame = {c['width'] * c['height'] / per / 1e6:.2f} Grays/s"
              f", frame equal: {same}", flush=True)
        for r in rts:
            r.destroy()
    rt.destroy()
    cam.destroy()
    sc.destroy()
    ctx.close()
