#!/usr/bin/env python3
"""Host-side enqueue rate of frames in flight against the GPU's rate (is a config host-bound?), and
what timing events around each frame cost (bench.py records a pair per frame).
    python tools/host_rate.py [c2|c3|c5] ...   (3 render targets on their own streams)"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from tools import ab_env  # noqa: E402
from raytracercuda_amd import beam, scenes  # noqa: E402


def run(ctx, cam, sc, rts, streams, c, n, evs):
    for i in range(6):
        ctx._check(cam.trace(c["eye"], scenes.IDENTITY, sc, rts[i % 3]))
    ctx.sync()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    t0 = time.perf_counter()
    for i in range(n):
        rec = evs and i % evs == 0
        if rec:
            ev[i][0].record(streams[i % 3])
        ctx._check(cam.trace(c["eye"], scenes.IDENTITY, sc, rts[i % 3]))
        if rec:
            ev[i][1].record(streams[i % 3])
    t1 = time.perf_counter()
    ctx.sync()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    return 1e3 * (t1 - t0) / n, 1e3 * (t2 - t0) / n


for name in sys.argv[1:] or ["c3"]:
    c = scenes.CONFIGS[name]
    ctx = ab_env.Context(device=0)
    sc = beam.IScene.create(ctx)
    keep = beam.upload_meshes(ctx, sc, scenes.scene(c["scene"]))
    sc.updateGPUScene()
    cam = beam.ICamera.create(ctx)
    cam.setInitialRays(c["width"], c["height"], *c["rays"])
    rts = [beam.IRenderTarget.createOffscreen(ctx, c["width"], c["height"]) for _ in range(3)]
    streams = [torch.cuda.Stream() for _ in range(3)]
    for r, s in zip(rts, streams):
        r.setStream(s.cuda_stream)
    for n in (20, 20, 200):
        for evs in (0, 1, 4):  # no events, a pair around every frame (bench.py), around every 4th
            enq, tot = run(ctx, cam, sc, rts, streams, c, n, evs)
            print(f"{name} {n} frames, events every {evs or '-'}: enqueue {enq:.4f} ms per frame, total {tot:.4f} ms "
                  f"per frame = {c['width'] * c['height'] / tot / 1e3:.0f} Mrays/s", flush=True)
    for r in rts:
        r.destroy()
    cam.destroy()
    sc.destroy()
    ctx.close()
