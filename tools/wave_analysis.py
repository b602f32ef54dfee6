#!/usr/bin/env python3
"""Per-wave traversal work of the trace kernel's pixel->lane mapping, from the CPU oracle's
per-ray counters (same traversal, same counts): SIMD efficiency = mean lane work / max lane work."""
import ctypes as C
import sys
import os
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import Oracle
from raytracercuda_amd import scenes

def main(scene="bunny", w=1920, h=1080, leaf=4, tile=8):
    o = Oracle()
    o.lib.orc_set_ray_stats.argtypes = [C.POINTER(C.c_uint32)]
    meshes = scenes.scene(scene)
    err, rays = o.camera_rays(w, h, *scenes.RAYS_1080)
    b = o.bvh_build(meshes, leaf)
    st = np.zeros((h * w, 2), np.uint32)
    o.lib.orc_set_ray_stats(st.ctypes.data_as(C.POINTER(C.c_uint32)))
    b.render(rays, scenes.BUNNY_EYE, scenes.IDENTITY)
    o.lib.orc_set_ray_stats(None)
    nodes = st[:, 0].reshape(h, w).astype(np.int64)
    tris = st[:, 1].reshape(h, w).astype(np.int64)
    # wave = tile x tile pixels (8x8 = 64 lanes)
    hh, ww = (h // tile) * tile, (w // tile) * tile
    def waves(a):
        return a[:hh, :ww].reshape(hh // tile, tile, ww // tile, tile).transpose(0, 2, 1, 3).reshape(-1, tile * tile)
    wn, wt = waves(nodes), waves(tris)
    cost = wn + wt  # crude: one loop iteration per node record or triangle
    print(f"{scene} {w}x{h} leaf={leaf}: rays {w*h}, mean nodes/ray {nodes.mean():.2f}, tris/ray {tris.mean():.2f}")
    print(f"  waves {wn.shape[0]}, mean(max lane nodes) {wn.max(1).mean():.2f}, mean(max lane tris) {wt.max(1).mean():.2f}")
    print(f"  SIMD efficiency nodes {wn.mean()/wn.max(1).mean():.3f}, tris {wt.mean()/max(wt.max(1).mean(),1e-9):.3f}")
    busy = cost.max(1)
    print(f"  waves with any hit-region work (>3 nodes): {(wn.max(1) > 3).sum()} ({(wn.max(1) > 3).mean()*100:.1f}%)")
    print(f"  sum over waves of max-lane iterations: {busy.sum()} ; hit rays {int((tris>0).sum())}")
    hit = tris > 0
    print(f"  rays with tri tests: nodes mean {nodes[hit].mean():.2f} max {nodes.max()}, tris mean {tris[hit].mean():.2f} max {tris.max()}")

if __name__ == "__main__":
    main(*(sys.argv[1:2] or ["bunny"]), leaf=int(sys.argv[2]) if len(sys.argv) > 2 else 4)
