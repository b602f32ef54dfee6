#!/usr/bin/env python3
"""Build time of a scene whose top Morton digit puts almost every key in one bucket: the bunny plus one
far triangle (the scene bounds grow ~1000x, the bunny falls into one top-level cell), so the first
build's k_bucket_sort takes its global (tiled, one-workgroup) path for that bucket and reports it; the
later builds of the scene sort with the three LSD passes. Compare BM_MSD_MAX_N=0 (LSD always)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools import ab_env  # noqa: E402
from raytracercuda_amd import beam, scenes  # noqa: E402

ctx = ab_env.Context(device=0)
bunny = scenes.load_mesh("bunny")
far = {"pos": np.array([100, 100, 100, 101, 100, 100, 100, 101, 100], np.float32),
       "nrm": np.zeros(9, np.float32), "idx": np.arange(3, dtype=np.uint32)}
for name, meshes in (("bunny", bunny), ("bunny+far", bunny + [far])):
    sc = beam.IScene.create(ctx)
    keep = beam.upload_meshes(ctx, sc, meshes)
    ms = [sc.updateGPUScene(stats=True)["build_ms"] for _ in range(12)]
    print(f"{name:12s} {sc.last_stats['num_tris']:8d} tris: builds 1-3 {ms[0]:.3f} {ms[1]:.3f} {ms[2]:.3f} ms, "
          f"median of the rest {np.median(ms[3:]):.3f} ms", flush=True)
    sc.destroy()
    del keep
ctx.close()
