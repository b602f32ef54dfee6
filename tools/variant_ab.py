#!/usr/bin/env python3
"""A/B of trace kernel variants on the bench camera: frames and counters compared bit for bit
against the first variant, median trace time per variant (HIP events on the context's stream).

    python tools/variant_ab.py [variants=6,10] [scenes=bunny,armadillo_proxy,merged_proxy] [iters=50]
Variants other than the product kernels need an A/B build: BEAM_HIP_LIB=<tools/build_ab.py out.so BM_TRACE_AB=1>.
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from raytracercuda_amd import beam, scenes
    from tools import ab_env
    variants = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "6,10").split(",")]
    names = (sys.argv[2] if len(sys.argv) > 2 else "bunny,armadillo_proxy,merged_proxy").split(",")
    iters = int(sys.argv[3]) if len(sys.argv) > 3 else 50
    stream = torch.cuda.current_stream()
    shadow = os.environ.get("AB_SHADOW") == "1"  # primary + one shadow ray per hit (fused)
    eye = scenes.FILLED_EYE if os.environ.get("AB_FILLED") == "1" else scenes.BUNNY_EYE  # filled view: 85 % hits
    ok_all = True
    for name in names:
        meshes = scenes.scene(name)
        ref = None
        for v in variants:
            os.environ["BM_TRACE_VARIANT"] = str(v)  # read by bm_context_create
            ctx = ab_env.Context(device=0, stream=stream.cuda_stream)
            scene = beam.IScene.create(ctx)
            keep = beam.upload_meshes(ctx, scene, meshes)
            scene.updateGPUScene()
            cam = beam.ICamera.create(ctx)
            ctx._check(cam.setInitialRays(1920, 1080, *scenes.RAYS_1080))
            rt = beam.IRenderTarget.createOffscreen(ctx, 1920, 1080)
            light = (0.0, 10.0, -10.0)
            if shadow:
                cnt = cam.traceShadowCounters(eye, scenes.IDENTITY, scene, rt, light)

                def frame():
                    return cam.traceShadow(eye, scenes.IDENTITY, scene, rt, light)
            else:
                cnt = cam.traceCounters(eye, scenes.IDENTITY, scene, rt)

                def frame():
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
            fr = rt.read()
            if shadow:
                fr["shadow"] = rt.readShadow()
            same = ""
            if ref is None:
                ref = (fr, cnt)
            else:
                eq = all(np.array_equal(fr[k].view(np.uint32), ref[0][k].view(np.uint32)) for k in fr)
                eqc = np.array_equal(cnt, ref[1])
                ok_all &= eq and eqc
                same = f" frame {'==' if eq else '!='} v{variants[0]}, counters {'==' if eqc else '!='}"
            print(f"{name:16s}{' +shadow' if shadow else ''} v{v:<3d} median {np.median(ms) * 1e3:7.1f} us min {min(ms) * 1e3:7.1f} us "
                  f"counters {cnt.tolist()}{same}", flush=True)
            rt.destroy()
            cam.destroy()
            scene.destroy()
            del keep
            ctx.close()
    print("ALL IDENTICAL" if ok_all else "MISMATCH", flush=True)
    return 0 if ok_all else 1


if __name__ == "__main__":
    sys.exit(main())
