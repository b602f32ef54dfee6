#!/usr/bin/env python3
"""Work estimate of wider BVH collapses (CPU, oracle): the LBVH's binary tree (BVH2 records from the
oracle) collapsed every 2 levels (BVH4, what the GPU traces) and every 3 levels (BVH8), traversed
nearest-first with the same culling, on a sample of rays of one view. Prints record visits, child box
tests and triangle tests per ray: the dependent steps a wider node would save and the box work it adds.

    python tools/wide_bvh_estimate.py [scene=armadillo_proxy] [view=filled|bench] [sample=20000]
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import Oracle  # noqa: E402
from raytracercuda_amd import scenes  # noqa: E402

LEAF, EMPTY = 0x80000000, 0xFFFFFFFF


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "armadillo_proxy"
    view = sys.argv[2] if len(sys.argv) > 2 else "filled"
    sample = int(sys.argv[3]) if len(sys.argv) > 3 else 20000
    o = Oracle()
    b = o.bvh_build(scenes.scene(name), 4, 2)
    rec, tris, _, _ = b.export()
    boxes = rec[:, :12].view(np.float32).reshape(-1, 2, 6)  # [node][child][lo xyz hi xyz]
    refs = rec[:, 12:14]
    tv = tris.view(np.float32).reshape(-1, 3, 4)
    err, rays = o.camera_rays(1920, 1080, *scenes.RAYS_1080)
    eye = np.float32(scenes.FILLED_EYE if view == "filled" else scenes.BUNNY_EYE)
    rng = np.random.default_rng(1)
    idx = rng.choice(rays.shape[0], sample, replace=False)

    def frontier(node, depth):
        """(box, ref) of the descendants `depth` binary levels below internal node `node`."""
        out = []
        for c in range(2):
            r = int(refs[node, c])
            if r == EMPTY:
                continue
            if depth > 1 and not (r & LEAF):
                out += frontier(r, depth - 1)
            else:
                out.append((boxes[node, c], r))
        return out

    for width, depth in ((4, 2), (8, 3)):
        cache = {}
        nodes = tests = ttests = 0
        for i in idx:
            d = rays[i].astype(np.float32)
            with np.errstate(divide="ignore", invalid="ignore", over="ignore"):
                inv = np.float32(1) / d
            tbest = np.float32(np.inf)
            stack = [(0, np.float32(-np.inf))]
            while stack:
                ref, tn0 = stack.pop()
                if tn0 > tbest:
                    continue
                if ref & LEAF:
                    first, cnt = ref & 0x07FFFFFF, ((ref >> 27) & 15) + 1
                    for k in range(first, first + cnt):
                        ttests += 1
                        v0, e1, e2 = tv[k, 0, :3], tv[k, 1, :3], tv[k, 2, :3]
                        p = np.cross(d, e2)
                        det = np.dot(e1, p)
                        if det == 0:
                            continue
                        s = eye - v0
                        u = np.dot(s, p) / det
                        q = np.cross(s, e1)
                        v = np.dot(d, q) / det
                        t = np.dot(e2, q) / det
                        if 0 <= u <= 1 and v >= 0 and u + v <= 1 and 0 < t < tbest:
                            tbest = np.float32(t)
                    continue
                nodes += 1
                if ref not in cache:
                    fr = frontier(ref, depth)
                    cache[ref] = (np.array([f[0] for f in fr], np.float32), [f[1] for f in fr])
                bx, rf = cache[ref]
                tests += len(rf)
                with np.errstate(invalid="ignore", over="ignore"):
                    tl = (bx[:, :3] - eye) * inv
                    th = (bx[:, 3:] - eye) * inv
                    tn = np.nanmax(np.minimum(tl, th), axis=1)
                    tf = np.nanmin(np.maximum(tl, th), axis=1)
                hit = (tn <= tf) & (tf >= 0) & (tn <= tbest)
                order = sorted((float(tn[j]), j) for j in np.nonzero(hit)[0])
                for tnj, j in reversed(order):
                    stack.append((rf[j], np.float32(tnj)))
        print(f"{name} {view} BVH{width}: record visits/ray {nodes / sample:.2f}, child box tests/ray {tests / sample:.1f}, "
              f"triangle tests/ray {ttests / sample:.2f}", flush=True)


if __name__ == "__main__":
    main()
