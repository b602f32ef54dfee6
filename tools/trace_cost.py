#!/usr/bin/env python3
"""Kernel-time decomposition experiments: empty scene (setup + writes only), camera looking away,
normal view; per trace variant.
Variants other than the product kernels need an A/B build: BEAM_HIP_LIB=<tools/build_ab.py out.so BM_TRACE_AB=1>.
"""
import os
import sys
import time
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools import ab_env  # noqa: E402
from raytracercuda_amd import beam, scenes  # noqa: E402


def timeit(ctx, cam, eye, orient, scene, rt, iters=50):
    for _ in range(5):
        ctx._check(cam.trace(eye, orient, scene, rt))
    ctx.sync()
    t0 = time.perf_counter()
    for _ in range(iters):
        ctx._check(cam.trace(eye, orient, scene, rt))
    ctx.sync()
    return (time.perf_counter() - t0) / iters * 1e3


for v in (sys.argv[1].split(",") if len(sys.argv) > 1 else ["0", "3"]):
    os.environ["BM_TRACE_VARIANT"] = v
    ctx = ab_env.Context(device=0)
    cam = beam.ICamera.create(ctx)
    ctx._check(cam.setInitialRays(1920, 1080, *scenes.RAYS_1080))
    rt = beam.IRenderTarget.createOffscreen(ctx, 1920, 1080)
    empty = beam.IScene.create(ctx)
    empty.updateGPUScene(stats=True)
    bunny = beam.IScene.create(ctx)
    keep = beam.upload_meshes(ctx, bunny, scenes.scene("bunny"))
    bunny.updateGPUScene(stats=True)
    away = np.eye(3, dtype=np.float32)
    away[2, 2] = -1.0  # look along -z: every ray misses the root box
    away[0, 0] = -1.0
    r = {
        "empty scene": timeit(ctx, cam, scenes.BUNNY_EYE, scenes.IDENTITY, empty, rt),
        "bunny, looking away": timeit(ctx, cam, scenes.BUNNY_EYE, away.reshape(9), bunny, rt),
        "bunny view": timeit(ctx, cam, scenes.BUNNY_EYE, scenes.IDENTITY, bunny, rt),
    }
    print(f"variant {v}: " + ", ".join(f"{k} {ms*1e3:.0f} us" for k, ms in r.items()), flush=True)
    rt.destroy(); cam.destroy(); empty.destroy(); bunny.destroy(); ctx.close()
