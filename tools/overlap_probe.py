#!/usr/bin/env python3
"""Frames in flight: whole-job primary-ray throughput with F render targets, each on its own HIP
stream (bm_rt_set_stream), tracing alternate frames of one scene, against F = 1 (every frame into
one target on the context stream).

    python tools/overlap_probe.py [scene] [frames] [F...]

With F > 1 consecutive frames are independent launches on different streams, so the next frame's
workgroups fill the CUs the previous frame's tail leaves idle. Prints one line per F.
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from raytracercuda_amd import beam, scenes
    from tools import ab_env
    name = sys.argv[1] if len(sys.argv) > 1 else "bunny"
    frames = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    fs = [int(a) for a in sys.argv[3:]] or [1, 2, 3]
    meshes = scenes.scene(name)
    torch.cuda.set_device(0)
    ctx = ab_env.Context(device=0)
    sc = beam.IScene.create(ctx)
    keep = beam.upload_meshes(ctx, sc, meshes)
    sc.updateGPUScene()
    cam = beam.ICamera.create(ctx)
    ctx._check(cam.setInitialRays(1920, 1080, *scenes.RAYS_1080))
    for F in fs:
        streams = [torch.cuda.Stream() for _ in range(F)] if F > 1 else [None]
        rts = []
        for st in streams:
            rt = beam.IRenderTarget.createOffscreen(ctx, 1920, 1080)
            if st is not None:
                rt.setStream(st.cuda_stream)
            rts.append(rt)

        def run(n):
            for i in range(n):
                ctx._check(cam.trace(scenes.BUNNY_EYE, scenes.IDENTITY, sc, rts[i % F]))

        run(10 * F)
        ctx.sync()
        reps = []
        for _ in range(3):
            t0 = time.perf_counter()
            run(frames)
            ctx.sync()
            reps.append((time.perf_counter() - t0) / frames * 1e3)
        ms = float(np.median(reps))
        hits = [int((rt.read(tri_id=False, t=False)["packed"] != 0xFF00).sum()) for rt in rts]
        print(f"{name:16s} F={F}: {ms * 1e3:7.1f} us/frame  {1920 * 1080 / ms / 1e3:8.0f} Mrays/s  hits {hits}",
              flush=True)
        for rt in rts:
            rt.destroy()
    cam.destroy()
    sc.destroy()
    del keep
    ctx.close()


if __name__ == "__main__":
    main()
