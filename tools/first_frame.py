#!/usr/bin/env python3
"""Latency of the first trace into a fresh render target vs later ones (HIP events on the context
stream), bunny 1080p: a render target made after others were destroyed, and one made fresh."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from tools import ab_env  # noqa: E402
from raytracercuda_amd import beam, scenes  # noqa: E402

st = torch.cuda.current_stream()
ctx = ab_env.Context(device=0, stream=st.cuda_stream)
sc = beam.IScene.create(ctx)
keep = beam.upload_meshes(ctx, sc, scenes.scene("bunny"))
sc.updateGPUScene()
cam = beam.ICamera.create(ctx)
cam.setInitialRays(1920, 1080, *scenes.RAYS_1080)


def timed(rt, n):
    out = []
    for _ in range(n):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        ctx._check(cam.trace(scenes.BUNNY_EYE, scenes.IDENTITY, sc, rt))
        b.record(st)
        torch.cuda.synchronize()
        out.append(round(a.elapsed_time(b) * 1e3))
    return out


for k in range(3):
    rt = beam.IRenderTarget.createOffscreen(ctx, 1920, 1080)
    t0 = time.perf_counter()
    print(f"target {k}: us per trace", timed(rt, 6), f"host {1e3 * (time.perf_counter() - t0):.1f} ms", flush=True)
    if k < 2:
        rt.read(rgb=True)
        rt.destroy()
