#!/usr/bin/env python3
"""Trace one scene N times with the current BM_TRACE_VARIANT (profiling driver)."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools import ab_env  # noqa: E402
from raytracercuda_amd import beam, scenes  # noqa: E402

scene_name = sys.argv[1] if len(sys.argv) > 1 else "bunny"
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 10
ctx = ab_env.Context(device=0)
scene = beam.IScene.create(ctx)
keep = beam.upload_meshes(ctx, scene, scenes.scene(scene_name))
scene.updateGPUScene(stats=True)
cam = beam.ICamera.create(ctx)
ctx._check(cam.setInitialRays(1920, 1080, *scenes.RAYS_1080))
rt = beam.IRenderTarget.createOffscreen(ctx, 1920, 1080)
for _ in range(iters):
    ctx._check(cam.trace(scenes.BUNNY_EYE, scenes.IDENTITY, scene, rt))
ctx.sync()
print("done")
