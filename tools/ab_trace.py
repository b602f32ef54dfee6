#!/usr/bin/env python3
"""Median primary-trace (and optionally shadow-pass) time of the current library build.

    python tools/ab_trace.py [scenes] [iters]        (BEAM_HIP_LIB=<other .so> to time another build)

Runs each scene at 1920x1080 with the bench camera; the trace is timed with HIP events on the
library's stream (torch's current stream handed to the context), median over `iters` frames,
interleaving nothing else. Prints one line per scene.
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from raytracercuda_amd import beam, scenes
    from tools import ab_env
    names = sys.argv[1].split(",") if len(sys.argv) > 1 else ["bunny", "armadillo_proxy"]
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    shadow = os.environ.get("AB_SHADOW") == "1"
    eye = scenes.FILLED_EYE if os.environ.get("AB_FILLED") == "1" else scenes.BUNNY_EYE  # filled view: 85 % hits
    stream = torch.cuda.current_stream()
    ctx = ab_env.Context(device=0, stream=stream.cuda_stream)
    tag = os.path.basename(os.environ.get("BEAM_HIP_LIB", "libbeam_hip.so"))
    for name in names:
        scene = beam.IScene.create(ctx)
        if name == "empty":  # no triangles: the per-pixel floor (ray setup + writes, no node fetch)
            meshes = []
        elif name == "onetri":  # one triangle outside the view: root fetch + miss for every ray
            meshes = [{"pos": np.float32([[50, 50, 50], [51, 50, 50], [50, 51, 50]]), "nrm": np.float32([[0, 0, 1]] * 3),
                       "idx": np.arange(3, dtype=np.uint32)}]
        else:
            meshes = scenes.scene(name)
        keep = beam.upload_meshes(ctx, scene, meshes)
        scene.updateGPUScene()
        cam = beam.ICamera.create(ctx)
        ctx._check(cam.setInitialRays(1920, 1080, *scenes.RAYS_1080))
        rt = beam.IRenderTarget.createOffscreen(ctx, 1920, 1080)
        light = (0.0, 10.0, -10.0)

        def frame():
            if shadow:
                return cam.traceShadow(eye, scenes.IDENTITY, scene, rt, light)
            return cam.trace(eye, scenes.IDENTITY, scene, rt)

        for _ in range(10):
            ctx._check(frame())
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
        for a, b in ev:
            a.record(stream)
            ctx._check(frame())
            b.record(stream)
        torch.cuda.synchronize()
        ms = [a.elapsed_time(b) for a, b in ev]
        print(f"{tag:24s} {name:16s} {'shadow' if shadow else 'primary':8s} median {np.median(ms) * 1e3:7.1f} us "
              f"min {min(ms) * 1e3:7.1f} us", flush=True)
        rt.destroy()
        cam.destroy()
        scene.destroy()
        del keep
    ctx.close()


if __name__ == "__main__":
    main()
