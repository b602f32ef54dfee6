"""BVH8 (BM_OPT_BVH8): 256-B records collapsed from the BVH2 records every three binary levels
(k_pack8) and the quad kernel with two children per lane (quad_visit8). Records bit-identical to the
oracle's width-8 build on every reachable slot, frames (ids, packed colours, t) and traversal
counters equal to the oracle's BVH8 traversal, fused shadow rays, refit, and the option's limits."""
import numpy as np
import pytest

from raytracercuda_amd import beam, scenes
from test_gpu_variants import check, expect, render

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not beam.ab_build(), reason="BVH8 is built into A/B builds only (BM_TRACE_AB=1)")]

LIGHT = (0.0, 10.0, -10.0)


@pytest.fixture
def ctx8():
    made = []

    def make(**kw):
        c = beam.Context(device=0, bvh_width=8, **kw)
        made.append(c)
        return c

    yield make
    for c in made:
        c.close()


@pytest.mark.parametrize("name,leaf", [("bunny", 4), ("suzanne", 1), ("f16", 16), ("armadillo_proxy", 4),
                                       ("merged_proxy", 4), ("f16", 4)])
def test_bvh8_records_bit_identical_to_oracle(ctx8, oracle, name, leaf):
    ctx = ctx8(leaf_size=leaf)
    meshes = scenes.scene(name)
    scene = beam.IScene.create(ctx)
    keep = beam.upload_meshes(ctx, scene, meshes)
    st = scene.updateGPUScene(stats=True)
    assert st["bvh_width"] == 8
    rec, tris, keys, perm = scene.export()
    orec, otris, okeys, operm = oracle.bvh_build(meshes, leaf, 8).export()
    assert rec.shape == orec.shape and rec.shape[1] == 64
    assert np.array_equal(keys, okeys) and np.array_equal(perm, operm) and np.array_equal(tris, otris)
    reach = beam.reachable_records(orec)
    assert np.array_equal(reach, beam.reachable_records(rec))
    assert np.array_equal(rec[reach], orec[reach]), f"{int((rec[reach] != orec[reach]).any(1).sum())} records differ"
    scene.destroy()
    del keep


@pytest.mark.parametrize("name,leaf,eye,size", [("bunny", 4, scenes.BUNNY_EYE, (1920, 1080)),
                                                ("armadillo_proxy", 4, scenes.FILLED_EYE, (640, 360)),
                                                ("suzanne", 1, (0.0, 0.0, -3.0), (480, 270)),
                                                ("f16", 16, (0.0, 0.0, -2.1), (500, 500)),
                                                ("merged_proxy", 4, scenes.BUNNY_EYE, (960, 540))])
def test_bvh8_frames_and_counters(ctx8, oracle, name, leaf, eye, size):
    ctx = ctx8(leaf_size=leaf)
    meshes = scenes.scene(name)
    w, h = size
    f, cnt = render(ctx, meshes, w, h, scenes.RAYS_1080, eye, scenes.IDENTITY)
    check(f, cnt, *expect(oracle, meshes, w, h, scenes.RAYS_1080, eye, scenes.IDENTITY, leaf, width=8))


def test_bvh8_frame_equals_bvh4(ctx8, oracle):
    """The closest hit does not depend on the node width: BVH8 and BVH4 frames agree bit for bit."""
    meshes = scenes.scene("armadillo_proxy")
    f8, c8 = render(ctx8(), meshes, 960, 540, scenes.RAYS_1080, scenes.FILLED_EYE, scenes.IDENTITY)
    c4ctx = beam.Context(device=0)
    f4, c4 = render(c4ctx, meshes, 960, 540, scenes.RAYS_1080, scenes.FILLED_EYE, scenes.IDENTITY)
    c4ctx.close()
    for k in f4:
        assert np.array_equal(f8[k].view(np.uint32), f4[k].view(np.uint32)), k
    assert c8[0] < c4[0] and c8[2] == c4[2]


@pytest.mark.parametrize("name", ["bunny", "merged_proxy"])
def test_bvh8_fused_shadow(ctx8, oracle, name):
    ctx = ctx8()
    meshes = scenes.scene(name)
    f, cnt = render(ctx, meshes, 640, 360, scenes.RAYS_1080, scenes.BUNNY_EYE, scenes.IDENTITY, light=LIGHT)
    check(f, cnt, *expect(oracle, meshes, 640, 360, scenes.RAYS_1080, scenes.BUNNY_EYE, scenes.IDENTITY, 4,
                          width=8, light=LIGHT))


def test_bvh8_refit(ctx8, oracle):
    ctx = ctx8()
    meshes = scenes.scene("bunny")
    scene = beam.IScene.create(ctx)
    keep = beam.upload_meshes(ctx, scene, meshes)
    scene.updateGPUScene()
    moved = [dict(m, pos=np.ascontiguousarray(np.asarray(m["pos"], np.float32).reshape(-1, 3) * np.float32(1.25)))
             for m in meshes]
    for mesh, m in zip(keep, moved):
        assert mesh.setVertexData(m["pos"], m["pos"].shape[0], 3, beam.VERTEX_DATA_POSITION) == 0
    scene.refitGPUScene()
    rec, tris, keys, perm = scene.export()
    ob = oracle.bvh_build(meshes, 4, 8).refit(moved)
    orec, otris, _, _ = ob.export()
    reach = beam.reachable_records(orec)
    assert np.array_equal(rec[reach], orec[reach]) and np.array_equal(tris, otris)
    scene.destroy()
    del keep


def test_bvh8_limits(ctx8):
    """BVH8 traces with the quad kernel only: the shadow queue and the trace variants are refused."""
    ctx = ctx8(shadow_queue=True)
    assert ctx.bvh_width == 8
    scene = beam.IScene.create(ctx)
    keep = beam.upload_meshes(ctx, scene, scenes.scene("f16"))
    scene.updateGPUScene()
    c = beam.ICamera.create(ctx)
    assert c.setInitialRays(64, 64, *scenes.RAYS_SQUARE) == 0
    rt = beam.IRenderTarget.createOffscreen(ctx, 64, 64)
    assert c.trace((0.0, 0.0, -2.1), scenes.IDENTITY, scene, rt) == 0  # primary rays: fine
    assert c.traceShadow((0.0, 0.0, -2.1), scenes.IDENTITY, scene, rt, LIGHT) == beam.ERROR_INVALID_PARAMETER
    rt.destroy()
    c.destroy()
    scene.destroy()
    del keep
