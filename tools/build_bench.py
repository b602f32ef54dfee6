#!/usr/bin/env python3
"""BVH build time (device, hipEvents inside bm_scene_build) per scene: median of repeated rebuilds."""
import os
import sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools import ab_env  # noqa: E402
from raytracercuda_amd import beam, scenes  # noqa: E402

ctx = ab_env.Context(device=0)
for name in (sys.argv[1].split(",") if len(sys.argv) > 1 else ["f16", "bunny", "armadillo_proxy", "merged_proxy"]):
    sc = beam.IScene.create(ctx)
    keep = beam.upload_meshes(ctx, sc, scenes.scene(name))
    ms = [sc.updateGPUScene(stats=True)["build_ms"] for _ in range(12)]
    st = sc.last_stats
    rf = [sc.refitGPUScene(stats=True)["build_ms"] for _ in range(12)]
    print(f"{name:16s} {st['num_tris']:8d} tris: build median {np.median(ms[2:]):.3f} ms (min {min(ms[2:]):.3f}, "
          f"first {ms[0]:.3f}); refit median {np.median(rf[2:]):.3f} ms; sort {st['sort_path']} front {st['fused_front']}",
          flush=True)
    sc.destroy()
