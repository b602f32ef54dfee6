#!/usr/bin/env python3
"""A/B the trace-kernel variants (BM_TRACE_VARIANT) on the GPU: time + bit-exact check vs variant 0.
Variants other than the product kernels need an A/B build: BEAM_HIP_LIB=<tools/build_ab.py out.so BM_TRACE_AB=1>.
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools import ab_env  # noqa: E402
from raytracercuda_amd import beam, scenes  # noqa: E402


def run(variant, scene_name, w, h, iters):
    v, _, scr = str(variant).partition(":")
    os.environ["BM_TRACE_VARIANT"] = v
    os.environ["BM_TRACE_SCRAMBLE"] = scr or "1"
    ctx = ab_env.Context(device=0)
    scene = beam.IScene.create(ctx)
    keep = beam.upload_meshes(ctx, scene, scenes.scene(scene_name))
    scene.updateGPUScene(stats=True)
    cam = beam.ICamera.create(ctx)
    ctx._check(cam.setInitialRays(w, h, *scenes.RAYS_1080))
    rt = beam.IRenderTarget.createOffscreen(ctx, w, h)
    for _ in range(5):
        ctx._check(cam.trace(scenes.BUNNY_EYE, scenes.IDENTITY, scene, rt))
    ctx.sync()
    t0 = time.perf_counter()
    for _ in range(iters):
        ctx._check(cam.trace(scenes.BUNNY_EYE, scenes.IDENTITY, scene, rt))
    ctx.sync()
    ms = (time.perf_counter() - t0) / iters * 1e3
    f = rt.read()
    rt.destroy(); cam.destroy(); scene.destroy(); ctx.close()
    del keep
    return ms, f


def main():
    variants = sys.argv[1].split(",") if len(sys.argv) > 1 else ["0", "2", "3", "4"]
    scenes_ = sys.argv[2].split(",") if len(sys.argv) > 2 else ["bunny", "armadillo_proxy"]
    for sn in scenes_:
        ref = None
        for v in variants:
            ms, f = run(v, sn, 1920, 1080, 50)
            same = "" if ref is None else (" identical" if all(np.array_equal(f[k], ref[k]) for k in f) else " DIFFERENT")
            if ref is None:
                ref = f
            print(f"{sn:16s} variant {v:5s}: {ms:.3f} ms/frame = {1920*1080/ms/1e3:.0f} Mrays/s{same}", flush=True)


if __name__ == "__main__":
    main()
