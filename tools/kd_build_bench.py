#!/usr/bin/env python3
"""Reference-mode (kd-tree) build time per scene: median build_ms (hipEvents inside bm_scene_build) of
repeated rebuilds. BM_KD_START=0 starts every walk at the root (A/B)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools import ab_env  # noqa: E402
from raytracercuda_amd import beam, scenes  # noqa: E402

ctx = ab_env.Context(device=0, reference_kd=True)
for name in (sys.argv[1].split(",") if len(sys.argv) > 1 else ["bunny", "armadillo_proxy", "merged_proxy"]):
    sc = beam.IScene.create(ctx)
    keep = beam.upload_meshes(ctx, sc, scenes.scene(name))
    ms = [sc.updateGPUScene(stats=True)["build_ms"] for _ in range(10)]
    print(f"{name:16s} {sc.last_stats['num_tris']:8d} tris: kd build median {np.median(ms[2:]):.3f} ms "
          f"(min {min(ms[2:]):.3f}, first {ms[0]:.3f})", flush=True)
    sc.destroy()
    del keep
ctx.close()
