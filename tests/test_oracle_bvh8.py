"""The oracle's BVH8 collapse (groundwork for a wider GPU node, DESIGN.md §5 "Next lever"): the same
LBVH binary tree collapsed every three levels into 256-B records, traversed nearest-first with
order_key8. A closest hit does not depend on the tree's width (the boxes are the same conservative
padded boxes), so every frame must equal the BVH4 oracle's bit for bit, with fewer record visits."""
import numpy as np
import pytest

from oracle import Oracle
from raytracercuda_amd import scenes


@pytest.mark.parametrize("name,w,h,eye", [("bunny", 256, 256, scenes.BUNNY_EYE), ("suzanne", 128, 128, (0.0, 0.0, -3.0)),
                                          ("f16", 160, 160, (0.0, 0.0, -2.1))])
def test_bvh8_frames_equal_bvh4(name, w, h, eye):
    o = Oracle()
    meshes = scenes.scene(name)
    err, rays = o.camera_rays(w, h, -1.0, 1.0, 1.0, -1.0, 1.0)
    b4 = o.bvh_build(meshes, 4, 4)
    b8 = o.bvh_build(meshes, 4, 8)
    p4, t4, d4, c4 = b4.render(rays, eye, scenes.IDENTITY, counters=True)
    p8, t8, d8, c8 = b8.render(rays, eye, scenes.IDENTITY, counters=True)
    assert np.array_equal(t4, t8) and np.array_equal(p4, p8) and np.array_equal(d4.view(np.uint32), d8.view(np.uint32))
    assert (t4 != 0xFFFFFFFF).sum() > 0
    assert c8[0] < c4[0], "BVH8 should visit fewer records"
    assert c8[1] == c4[1] or abs(int(c8[1]) - int(c4[1])) <= 0.05 * int(c4[1])
    assert c8[2] == c4[2]


def test_bvh8_record_layout():
    o = Oracle()
    b8 = o.bvh_build(scenes.scene("f16"), 4, 8)
    rec, tris, keys, perm = b8.export()
    assert rec.shape[1] == 64
    root = rec[0]
    refs = root[48:56]
    used = refs != 0xFFFFFFFF
    assert used.sum() >= 2
    lo = root[:24].view(np.float32).reshape(3, 8)
    hi = root[24:48].view(np.float32).reshape(3, 8)
    assert np.all(lo[:, used] <= hi[:, used]) and np.all(np.isnan(lo[:, ~used]))
    assert np.all(root[56:] == 0)
