#!/usr/bin/env python3
"""Tree-quality experiment (CPU, oracle): the per-ray work and the heaviest 8x8 tile of a BVH from
another builder, traversed exactly like the LBVH (same collapse, BVH4 packing and traversal).

    python tools/tree_quality.py [scene] [width]

Builders compared: the Karras LBVH (what the GPU builds) and a full-sweep SAH binary tree
(top-down, every split position on every axis) — the usual quality reference.
"""
import ctypes as C
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle.oracle import Oracle, OrcBVH, OrcMeshes  # noqa: E402
from raytracercuda_amd import scenes  # noqa: E402

LEAF = 0x80000000


def tri_boxes(meshes):
    lo, hi = [], []
    for m in meshes:
        p = np.asarray(m["pos"], np.float32)[np.asarray(m["idx"], np.int64).reshape(-1, 3)]
        lo.append(p.min(1))
        hi.append(p.max(1))
    return np.concatenate(lo), np.concatenate(hi)


def area(lo, hi):
    e = np.maximum(hi - lo, 0)
    return e[..., 0] * e[..., 1] + e[..., 1] * e[..., 2] + e[..., 2] * e[..., 0]


def sah_tree(lo, hi, max_full=4096, bins=64):
    """Top-down SAH: full sweep for segments <= max_full, binned (64 bins) above. Returns
    (perm, lch, rch) with internal nodes numbered in creation order (root 0)."""
    n = lo.shape[0]
    cen = (lo + hi) * 0.5
    perm = np.arange(n, dtype=np.int64)
    lch = np.zeros(max(n - 1, 1), np.uint32)
    rch = np.zeros(max(n - 1, 1), np.uint32)
    next_id = [0]

    def new_node():
        i = next_id[0]
        next_id[0] += 1
        return i

    # stack of (segment start, end, node id to fill, which side of parent)
    root = new_node()
    stack = [(0, n, root)]
    while stack:
        s, e, node = stack.pop()
        idx = perm[s:e]
        k = e - s
        best = None
        if k <= max_full:
            for ax in range(3):
                order = np.argsort(cen[idx, ax], kind="stable")
                ids = idx[order]
                pl = np.minimum.accumulate(lo[ids]), np.maximum.accumulate(hi[ids])
                sl = np.minimum.accumulate(lo[ids][::-1])[::-1], np.maximum.accumulate(hi[ids][::-1])[::-1]
                cl = area(pl[0][:-1], pl[1][:-1]) * np.arange(1, k)
                cr = area(sl[0][1:], sl[1][1:]) * np.arange(k - 1, 0, -1)
                c = cl + cr
                j = int(np.argmin(c))
                if best is None or c[j] < best[0]:
                    best = (c[j], ids, j + 1)
        else:
            cmin, cmax = cen[idx].min(0), cen[idx].max(0)
            for ax in range(3):
                ext = cmax[ax] - cmin[ax]
                if ext <= 0:
                    continue
                b = np.minimum(((cen[idx, ax] - cmin[ax]) / ext * bins).astype(np.int64), bins - 1)
                cnt = np.bincount(b, minlength=bins)
                blo = np.full((bins, 3), np.inf, np.float32)
                bhi = np.full((bins, 3), -np.inf, np.float32)
                np.minimum.at(blo, b, lo[idx])
                np.maximum.at(bhi, b, hi[idx])
                plo, phi = np.minimum.accumulate(blo), np.maximum.accumulate(bhi)
                slo, shi = np.minimum.accumulate(blo[::-1])[::-1], np.maximum.accumulate(bhi[::-1])[::-1]
                nl = np.cumsum(cnt)[:-1]
                nr = k - nl
                c = area(plo[:-1], phi[:-1]) * nl + area(slo[1:], shi[1:]) * nr
                c = np.where((nl > 0) & (nr > 0), c, np.inf)
                j = int(np.argmin(c))
                if np.isfinite(c[j]) and (best is None or c[j] < best[0]):
                    order = np.argsort(b, kind="stable")
                    best = (c[j], idx[order], int(nl[j]))
            if best is None:  # all centroids equal: split in half
                best = (0, idx, k // 2)
        _, ids, split = best
        perm[s:e] = ids
        m = s + split
        for side, (a, z) in enumerate(((s, m), (m, e))):
            if z - a == 1:
                ref = a | LEAF
            else:
                ref = new_node()
                stack.append((a, z, ref))
            if side == 0:
                lch[node] = ref
            else:
                rch[node] = ref
    return perm.astype(np.uint32), lch, rch


def tile_stats(o, bvh, rays, eye, orient, W, H):
    per = np.zeros(2 * W * H, np.uint32)
    o.lib.orc_set_ray_stats(per.ctypes.data_as(C.POINTER(C.c_uint32)))
    packed, tri, t, cnt = bvh.render(rays, eye, orient, counters=True)
    o.lib.orc_set_ray_stats(None)
    nodes = per[0::2].reshape(H, W).astype(np.float64)
    tris = per[1::2].reshape(H, W).astype(np.float64)
    cost = (nodes + 0.5 * tris).reshape(H // 8, 8, W // 8, 8).max(axis=(1, 3))
    return tri, cnt, cost


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "bunny"
    width = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    o = Oracle()
    lib = o.lib
    lib.orc_bvh_build_tree.argtypes = [C.POINTER(type(OrcMeshes([]).arr[0])), C.c_uint32, C.c_uint32, C.c_uint32,
                                       C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]
    lib.orc_bvh_build_tree.restype = C.c_void_p
    meshes = scenes.scene(name)
    om = OrcMeshes(meshes)
    W, H = 1920, 1080
    err, rays = o.camera_rays(W, H, *scenes.RAYS_1080)
    eye, orient = (scenes.FILLED_EYE if os.environ.get("TQ_FILLED") else scenes.BUNNY_EYE), scenes.IDENTITY
    lb = o.bvh_build(om, 4, width)
    tri0, c0, cost0 = tile_stats(o, lb, rays, eye, orient, W, H)
    print(f"{name} LBVH W{width}: nodes/ray {c0[0] / rays.shape[0]:.2f} tris/ray {c0[1] / rays.shape[0]:.2f} "
          f"tile max {cost0.max():.0f} top10 {np.sort(cost0.ravel())[-10:].mean():.0f} sum {cost0.sum() / 1e3:.0f}K")
    t0 = time.time()
    lo, hi = tri_boxes(meshes)
    perm, lch, rch = sah_tree(lo, hi)
    print(f"SAH tree built in {time.time() - t0:.1f} s")
    u32 = lambda a: np.ascontiguousarray(a, np.uint32).ctypes.data_as(C.POINTER(C.c_uint32))  # noqa: E731
    b = OrcBVH.__new__(OrcBVH)
    b.lib, b.om, b.width = lib, om, width
    b.h = lib.orc_bvh_build_tree(om.arr, om.count, 4, width, u32(perm), u32(lch), u32(rch))
    b.n = lib.orc_bvh_num_tris(b.h)
    b.num_records = lib.orc_bvh_num_records(b.h)
    b.record_words = lib.orc_bvh_record_words(b.h)
    tri1, c1, cost1 = tile_stats(o, b, rays, eye, orient, W, H)
    print(f"{name} SAH  W{width}: nodes/ray {c1[0] / rays.shape[0]:.2f} tris/ray {c1[1] / rays.shape[0]:.2f} "
          f"tile max {cost1.max():.0f} top10 {np.sort(cost1.ravel())[-10:].mean():.0f} sum {cost1.sum() / 1e3:.0f}K")
    print("same frame:", np.array_equal(tri0, tri1))


if __name__ == "__main__":
    main()
