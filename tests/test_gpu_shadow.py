"""GPU parity of the shadow pass: one any-hit shadow ray per primary hit toward a
point light, origin eye + dir * (t * 0.9999f), segment to the light, shadowed when 0 < t_s < 1.

The reference has no shadow rays, so the semantics are this build's; the checker is
the oracle's any-hit LBVH traversal (orc_bvh_shadow, same order, so the counters match too), itself
pinned to the exhaustive fixture tests/golden/views/bunny_256_shadow.npz (CPU test). Bar: the
shadow plane is bit-exact; the primary planes are unchanged by the shadow pass.
"""
import numpy as np
import pytest

from golden_io import view
from gpu_util import gpu_build, oracle_shadow, shadow_frame
from raytracercuda_amd import beam, multigpu, scenes

pytestmark = pytest.mark.gpu

C5_LIGHT = (0.0, 10.0, -10.0)


def build(ctx, meshes):
    scene, keep, _ = gpu_build(ctx, meshes)
    return scene, keep


def test_shadow_golden_bunny_256(ctx):
    g = view("bunny_256_shadow")
    scene, keep = build(ctx, scenes.load_mesh("bunny"))
    plain = None
    for k, light in enumerate(g["lights"]):
        f, _ = shadow_frame(ctx, scene, 256, 256, scenes.RAYS_SQUARE, scenes.BUNNY_EYE, scenes.IDENTITY, light)
        assert np.array_equal(np.flatnonzero(f["shadow"]), g[f"pixels_{k}"])
        if plain is None:
            c = beam.ICamera.create(ctx)
            assert c.setInitialRays(256, 256, *scenes.RAYS_SQUARE) == 0
            rt = beam.IRenderTarget.createOffscreen(ctx, 256, 256)
            assert c.trace(scenes.BUNNY_EYE, scenes.IDENTITY, scene, rt) == 0
            plain = {k2: v.reshape(-1) for k2, v in rt.read().items()}
            rt.destroy()
            c.destroy()
        for key in ("packed", "tri_id", "t"):  # the shadow pass leaves the primary planes alone
            assert np.array_equal(f[key], plain[key])
    scene.destroy()


@pytest.mark.parametrize("name,light", [("bunny", (3.0, 2.0, 0.0)), ("f16", C5_LIGHT), ("suzanne", (-2.0, 3.0, -4.0))])
def test_shadow_counters_match_oracle(ctx, oracle, name, light):
    meshes = scenes.load_mesh(name)
    eye = {"bunny": scenes.BUNNY_EYE, "f16": (0.0, 0.0, -2.1), "suzanne": (0.0, 0.0, -3.0)}[name]
    scene, keep = build(ctx, meshes)
    f, cnt = shadow_frame(ctx, scene, 200, 150, scenes.RAYS_SQUARE, eye, scenes.IDENTITY, light, counters=True)
    packed, tri, t, sh, ocnt = oracle_shadow(oracle, meshes, 200, 150, scenes.RAYS_SQUARE, eye, scenes.IDENTITY,
                                             light)
    assert np.array_equal(f["tri_id"], tri)
    assert np.array_equal(f["shadow"], sh)
    assert list(map(int, cnt[3:])) == list(map(int, ocnt)), (cnt, ocnt)
    assert int(cnt[2]) == int((tri != 0xFFFFFFFF).sum())
    scene.destroy()


@pytest.mark.parametrize("ntri", [1, 2, 5, 17])
def test_shadow_tiny_scenes_against_exhaustive(ctx, oracle, ntri):
    rng = np.random.default_rng(100 + ntri)
    pos = rng.uniform(-1, 1, (3 * ntri, 3)).astype(np.float32)
    pos[:, 2] = rng.uniform(0.0, 2.0, 3 * ntri).astype(np.float32)
    meshes = [{"pos": pos, "nrm": np.tile(np.float32([0, 0, 1]), (3 * ntri, 1)),
               "idx": np.arange(3 * ntri, dtype=np.uint32)}]
    light = (0.2, 0.3, 4.0)
    eye = (0.0, 0.0, -2.0)
    scene, keep = build(ctx, meshes)
    f, _ = shadow_frame(ctx, scene, 37, 29, scenes.RAYS_SQUARE, eye, scenes.IDENTITY, light)
    err, rays = oracle.camera_rays(37, 29, *scenes.RAYS_SQUARE)
    _, tri, t = oracle.brute_render(meshes, rays, eye, scenes.IDENTITY)
    assert np.array_equal(f["tri_id"], tri)
    assert np.array_equal(f["shadow"], oracle.brute_shadow(meshes, rays, eye, scenes.IDENTITY, light, tri, t))
    scene.destroy()


def test_shadow_band_partition_reassembles(ctx):
    scene, keep = build(ctx, scenes.load_mesh("bunny"))
    w, h, bh = 96, 70, 16
    full, _ = shadow_frame(ctx, scene, w, h, scenes.RAYS_1080, scenes.BUNNY_EYE, scenes.IDENTITY, C5_LIGHT)
    cam = beam.ICamera.create(ctx)
    assert cam.setInitialRays(w, h, *scenes.RAYS_1080) == 0
    for world in (2, 3):
        rows = multigpu.rows_per_rank(h, bh, world)
        parts = []
        for r in range(world):
            rt = beam.IRenderTarget.createOffscreen(ctx, w, rows)
            assert cam.traceShadowBands(scenes.BUNNY_EYE, scenes.IDENTITY, scene, rt, bh, world, r, C5_LIGHT) == 0
            parts.append(np.stack([rt.readShadow().astype(np.uint32)]))
            rt.destroy()
        frame = multigpu.reassemble_np(np.stack(parts), h, bh)[0]
        assert np.array_equal(frame.reshape(-1), full["shadow"].astype(np.uint32))
    cam.destroy()
    scene.destroy()


def test_shadow_errors(ctx):
    scene, keep = build(ctx, scenes.load_mesh("suzanne"))
    cam = beam.ICamera.create(ctx)
    assert cam.setInitialRays(32, 32) == 0
    rt = beam.IRenderTarget.createOffscreen(ctx, 32, 32)
    with pytest.raises(beam.BeamError):
        rt.readShadow()  # no shadow trace yet
    assert cam.traceShadow((0, 0, -3), scenes.IDENTITY, scene, rt, (np.nan, 0, 0)) == beam.ERROR_INVALID_PARAMETER
    empty = beam.IScene.create(ctx)
    empty.updateGPUScene()
    assert cam.traceShadow((0, 0, -3), scenes.IDENTITY, empty, rt, C5_LIGHT) == 0
    assert not rt.readShadow().any()
    assert (rt.read()["tri_id"] == 0xFFFFFFFF).all()
    for s in (empty, scene):
        s.destroy()
    rt.destroy()
    cam.destroy()


def test_shadow_queue_mode_matches_fused(oracle):
    """The wavefront form (hit pixels compacted into a queue, separate persistent pass) gives the same
    shadow plane and the same traversal counters as the fused form."""
    meshes = scenes.load_mesh("bunny")
    out = []
    for queue in (False, True):
        c = beam.Context(device=0, shadow_queue=queue)
        scene, keep = build(c, meshes)
        f, cnt = shadow_frame(c, scene, 640, 360, scenes.RAYS_1080, scenes.BUNNY_EYE, scenes.IDENTITY, C5_LIGHT,
                              counters=True)
        f2, _ = shadow_frame(c, scene, 640, 360, scenes.RAYS_1080, scenes.BUNNY_EYE, scenes.IDENTITY, C5_LIGHT)
        assert np.array_equal(f["shadow"], f2["shadow"])
        out.append((f, cnt))
        scene.destroy()
        c.close()
    (fa, ca), (fb, cb) = out
    assert np.array_equal(fa["shadow"], fb["shadow"])
    assert np.array_equal(fa["tri_id"], fb["tri_id"])
    assert list(map(int, ca)) == list(map(int, cb))
    packed, tri, t, sh, ocnt = oracle_shadow(oracle, meshes, 640, 360, scenes.RAYS_1080, scenes.BUNNY_EYE,
                                             scenes.IDENTITY, C5_LIGHT)
    assert np.array_equal(fa["shadow"], sh)
