#!/usr/bin/env python3
"""Hashed-grid reference mode (Hash.cu) trace time on a config's frame, HIP events over a few traces.
    python tools/hash_time.py [c2|c3|...] ..."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from tools import ab_env  # noqa: E402
from raytracercuda_amd import beam, scenes  # noqa: E402

st = torch.cuda.current_stream()
for name in sys.argv[1:] or ["c2"]:
    c = scenes.CONFIGS[name]
    ctx = ab_env.Context(device=0, stream=st.cuda_stream, reference_hash=True)
    sc = beam.IScene.create(ctx)
    keep = beam.upload_meshes(ctx, sc, scenes.scene(c["scene"]))
    b = [sc.updateGPUScene(stats=True)["build_ms"] for _ in range(2)]
    cam = beam.ICamera.create(ctx)
    cam.setInitialRays(c["width"], c["height"], *c["rays"])
    rt = beam.IRenderTarget.createOffscreen(ctx, c["width"], c["height"])
    ctx._check(cam.trace(c["eye"], scenes.IDENTITY, sc, rt))
    a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(st)
    for _ in range(3):
        ctx._check(cam.trace(c["eye"], scenes.IDENTITY, sc, rt))
    e.record(st)
    torch.cuda.synchronize()
    ms = a.elapsed_time(e) / 3
    hits = int((rt.read()["tri_id"] != 0xFFFFFFFF).sum())
    print(f"{name} hashed grid: build {b[-1]:.3f} ms, trace {ms:.3f} ms = {c['width'] * c['height'] / ms / 1e3:.1f} "
          f"Mrays/s, hits {hits}", flush=True)
    rt.destroy()
    cam.destroy()
    sc.destroy()
    ctx.close()
