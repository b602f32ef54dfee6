"""Reference mode (BM_OPT_REFERENCE_KD) on one config, for rocprofv3 --kernel-trace --stats:
builds the kd-tree BUILDS times (build_ms of each printed) and traces FRAMES frames.

    python tools/prof_refmode.py [config] [builds] [frames]
"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    import torch

    from raytracercuda_amd import beam, scenes
    from tools import ab_env
    name = sys.argv[1] if len(sys.argv) > 1 else "c2"
    builds = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    frames = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    c = scenes.CONFIGS[name]
    stream = torch.cuda.Stream()
    ctx = ab_env.Context(device=0, stream=stream.cuda_stream, reference_kd=True)
    sc = beam.IScene.create(ctx)
    keep = beam.upload_meshes(ctx, sc, scenes.scene(c["scene"]))
    for i in range(builds):
        t0 = time.perf_counter()
        ms = sc.updateGPUScene(stats=True)["build_ms"]
        print(f"build {i}: events {ms:.3f} ms, host wall {1e3 * (time.perf_counter() - t0):.3f} ms", flush=True)
    cam = beam.ICamera.create(ctx)
    ctx._check(cam.setInitialRays(c["width"], c["height"], *c["rays"]))
    rt = beam.IRenderTarget.createOffscreen(ctx, c["width"], c["height"])
    for _ in range(frames):
        ctx._check(cam.trace(c["eye"], scenes.IDENTITY, sc, rt))
    torch.cuda.synchronize()
    print("kd stats (leaves, face refs):", sc.kdStats(), flush=True)
    rt.destroy()
    cam.destroy()
    sc.destroy()
    del keep
    ctx.close()


if __name__ == "__main__":
    main()
