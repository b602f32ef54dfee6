"""Reference mode (BM_OPT_REFERENCE_KD): the reference's own kd-tree build and march on the GPU.

Bar: every pixel — the early-out pixels included, where the reference returns a farther triangle than
the closest hit — equals the reference framebuffer: packed colour and triangle id bit-exact, t
bit-exact (within 1e-5 is the contract), against the golden frames of the kd restatement
(tests/golden/views, pinned to the SURVEY §8(c) known answers) and against the oracle's kd march on
views no fixture covers. The tree's content is checked through its statistics (face references
stored, faces dropped by the 256-face cap, largest leaf) against orc_kd_stats.
"""
import numpy as np
import pytest

from gpu_util import kd_frame
from raytracercuda_amd import beam, scenes

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def kctx():
    c = beam.Context(device=0, reference_kd=True)
    yield c
    c.close()


def test_reference_mode_sweep_and_merged_scene_vs_oracle(kctx, oracle):
    """Views without a fixture: the seeded camera sweep (bunny) and the 1.1M-triangle merged proxy,
    where the 256-face cap drops faces."""
    eyes, orients = scenes.sweep_views()
    meshes = scenes.load_mesh("bunny")
    err, rays = oracle.camera_rays(96, 96, *scenes.RAYS_SQUARE)
    for k in (0, 5, 11):
        f, _ = kd_frame(kctx, meshes, 96, 96, scenes.RAYS_SQUARE, eyes[k], orients[k])
        packed, tri, t = oracle.kd_render(meshes, rays, eyes[k], orients[k])
        assert np.array_equal(f["tri_id"], tri) and np.array_equal(f["packed"], packed)
        assert np.array_equal(f["t"], t)
    merged = scenes.scene("merged_proxy")
    err, rays = oracle.camera_rays(320, 180, *scenes.RAYS_1080)
    f, st = kd_frame(kctx, merged, 320, 180, scenes.RAYS_1080, scenes.BUNNY_EYE, scenes.IDENTITY)
    packed, tri, t, ost = oracle.kd_render(merged, rays, scenes.BUNNY_EYE, scenes.IDENTITY, stats=True)
    assert np.array_equal(f["tri_id"], tri) and np.array_equal(f["packed"], packed) and np.array_equal(f["t"], t)
    assert int(st[2]) == int(ost[3]) > 0  # the cap drops the same number of faces
    assert int(st[1]) == int(ost[2])


def test_reference_mode_limits(kctx):
    scene = beam.IScene.create(kctx)
    keep = beam.upload_meshes(kctx, scene, scenes.load_mesh("suzanne"))
    scene.updateGPUScene()
    cam = beam.ICamera.create(kctx)
    assert cam.setInitialRays(64, 48) == 0
    rt = beam.IRenderTarget.createOffscreen(kctx, 64, 48)
    assert cam.traceShadow((0, 0, -3), scenes.IDENTITY, scene, rt, (0, 10, -10)) == beam.ERROR_INVALID_PARAMETER
    with pytest.raises(beam.BeamError):
        scene.refitGPUScene()
    with pytest.raises(beam.BeamError):
        scene.export()
    empty = beam.IScene.create(kctx)
    empty.updateGPUScene()
    assert cam.trace((0, 0, -3), scenes.IDENTITY, empty, rt) == 0
    assert (rt.read()["tri_id"] == 0xFFFFFFFF).all()
    for s in (scene, empty):
        s.destroy()
    rt.destroy()
    cam.destroy()


def test_reference_mode_zero_direction_components_and_eye_on_split_planes(kctx, oracle):
    """Rays with an exactly zero direction component (1/dir infinite, NaN slab terms possible) from
    eyes on the world box's split planes: the march replays those chains level by level, as the
    reference does, and must still equal the kd oracle on every pixel."""
    meshes = scenes.load_mesh("suzanne")
    err, rays = oracle.camera_rays(64, 48, *scenes.RAYS_SQUARE)
    # orient rows set to zero: dir.x (or dir.y) == 0 for every ray
    flat_x = np.array([0, 0, 0, 0, 1, 0, 1, 0, 0], np.float32)  # column-major: row 0 all zero
    flat_y = np.array([1, 0, 0, 0, 0, 0, 0, 1, 1], np.float32)
    for eye, orient in [((0.0, 0.0, -3.0), flat_x), ((0.0, 0.0, -3.0), flat_y), ((15.0, 0.0, -3.0), flat_x),
                        ((0.0, 7.5, 0.0), flat_y), ((0.0, 0.0, -3.0), scenes.IDENTITY)]:
        f, _ = kd_frame(kctx, meshes, 64, 48, scenes.RAYS_SQUARE, eye, orient)
        packed, tri, t = oracle.kd_render(meshes, rays, eye, orient)
        assert np.array_equal(f["tri_id"], tri) and np.array_equal(f["packed"], packed)
        assert np.array_equal(f["t"].view(np.uint32), t.view(np.uint32))


@pytest.mark.parametrize("caps", [{"kd_lq_cap": 3}, {"kd_queue_cap": 40}, {"kd_lq_cap": 5, "kd_queue_cap": 1}])
def test_reference_mode_split_descent_queue_overflow(kctx, oracle, caps):
    """The split build (k_kd_top + k_kd_sub) with queues too small for the work: nodes that find the
    workgroup's LDS queue full are walked on by their lane, items that find the global queue full by
    the flushing lane. The tree (stats) and the frame must not change."""
    for k, v in caps.items():  # test hooks (bm_context_set_param)
        kctx.set_param(k, v)
    meshes = scenes.load_mesh("bunny")
    err, rays = oracle.camera_rays(128, 96, *scenes.RAYS_1080)
    f, st = kd_frame(kctx, meshes, 128, 96, scenes.RAYS_1080, scenes.BUNNY_EYE, scenes.IDENTITY)
    packed, tri, t, ost = oracle.kd_render(meshes, rays, scenes.BUNNY_EYE, scenes.IDENTITY, stats=True)
    assert np.array_equal(f["tri_id"], tri) and np.array_equal(f["packed"], packed) and np.array_equal(f["t"], t)
    assert int(st[1]) == int(ost[2]) and int(st[2]) == int(ost[3])
    assert (tri != 0xFFFFFFFF).sum() > 0


@pytest.mark.parametrize("variant", [2, 1])
def test_reference_mode_march_variants(oracle, variant):
    """The one-box march steps (BM_PARAM_KD_MARCH 2) and the lane-per-ray leaves (1) give the kd
    oracle's frames as the default (3: child-box steps) does — a silhouette view with grazing rays and
    a view whose rays have an exactly zero direction component (chain replay lanes)."""
    ctx = beam.Context(device=0, reference_kd=True, params={"kd_march": variant})
    try:
        meshes = scenes.load_mesh("bunny")
        err, rays = oracle.camera_rays(160, 120, *scenes.RAYS_1080)
        f, _ = kd_frame(ctx, meshes, 160, 120, scenes.RAYS_1080, scenes.BUNNY_EYE, scenes.IDENTITY)
        packed, tri, t = oracle.kd_render(meshes, rays, scenes.BUNNY_EYE, scenes.IDENTITY)
        assert np.array_equal(f["tri_id"], tri) and np.array_equal(f["packed"], packed) and np.array_equal(f["t"], t)
        flat_x = np.array([0, 0, 0, 0, 1, 0, 1, 0, 0], np.float32)
        err, rays = oracle.camera_rays(64, 48, *scenes.RAYS_SQUARE)
        f, _ = kd_frame(ctx, meshes, 64, 48, scenes.RAYS_SQUARE, (0.0, 0.0, -3.0), flat_x)
        packed, tri, t = oracle.kd_render(meshes, rays, (0.0, 0.0, -3.0), flat_x)
        assert np.array_equal(f["tri_id"], tri) and np.array_equal(f["packed"], packed) and np.array_equal(f["t"], t)
    finally:
        ctx.close()


@pytest.mark.parametrize("variant", [None, 2])
def test_reference_mode_filled_view_vs_oracle(oracle, variant):
    """The filled view (armadillo proxy, 85.5 % of pixels hit, ~120 face tests per ray): most lanes
    record several leaves before the wave's leaf round, and a round whose first leaf has no hit moves
    the lane's next recorded leaf up — the speculative path the silhouette views exercise least. Every
    pixel equals the kd oracle, with the default march and with one-box steps (BM_PARAM_KD_MARCH 2)."""
    params = {} if variant is None else {"kd_march": variant}
    ctx = beam.Context(device=0, reference_kd=True, params=params)
    try:
        c = scenes.CONFIGS["filled"]
        meshes = scenes.scene(c["scene"])
        err, rays = oracle.camera_rays(384, 216, *c["rays"])
        f, _ = kd_frame(ctx, meshes, 384, 216, c["rays"], c["eye"], scenes.IDENTITY)
        packed, tri, t = oracle.kd_render(meshes, rays, c["eye"], scenes.IDENTITY)
        assert (tri != 0xFFFFFFFF).mean() > 0.8
        assert np.array_equal(f["tri_id"], tri), f"{int((f['tri_id'] != tri).sum())} ids differ"
        assert np.array_equal(f["packed"], packed) and np.array_equal(f["t"], t)
    finally:
        ctx.close()


def test_reference_mode_full_c3_frame_vs_oracle(oracle):
    """reference mode at the headline size — the armadillo proxy (278,520 triangles) at
    1920x1080 from the bench eye — every pixel (triangle id, packed colour, t bits) against the oracle's
    restatement of the reference's kd build and first-hit-leaf march."""
    ctx = beam.Context(device=0, reference_kd=True)
    try:
        c = scenes.CONFIGS["c3"]
        meshes = scenes.scene(c["scene"])
        err, rays = oracle.camera_rays(c["width"], c["height"], *c["rays"])
        f, st = kd_frame(ctx, meshes, c["width"], c["height"], c["rays"], c["eye"], scenes.IDENTITY)
        packed, tri, t, ost = oracle.kd_render(meshes, rays, c["eye"], scenes.IDENTITY, stats=True)
        assert (tri != 0xFFFFFFFF).sum() > 100000
        assert np.array_equal(f["tri_id"], tri), f"{int((f['tri_id'] != tri).sum())} ids differ"
        assert np.array_equal(f["packed"], packed)
        assert np.array_equal(f["t"].view(np.uint32), t.view(np.uint32))
        assert int(st[1]) == int(ost[2]) and int(st[2]) == int(ost[3])  # face references stored / dropped
    finally:
        ctx.close()


def test_reference_mode_leaf_limit_is_reported_not_built(oracle):
    """a build with more kd leaves than it accepts (BM_PARAM_KD_MAX_LEAVES lowered from 2^25 as a
    test hook; the bunny has 16,742) writes no tree — the leaf-side kernels see the device count above their
    capacity and stay idle — and the first trace reports BM_ERROR_GPU_ALLOC_FAIL and leaves the scene
    unbuilt. With the limit restored the same scene builds and traces the oracle's frame."""
    ctx = beam.Context(device=0, reference_kd=True, params={"kd_max_leaves": 1000})
    try:
        meshes = scenes.load_mesh("bunny")
        scene = beam.IScene.create(ctx)
        keep = beam.upload_meshes(ctx, scene, meshes)
        scene.updateGPUScene()  # the count lives on the device: the build itself succeeds
        cam = beam.ICamera.create(ctx)
        assert cam.setInitialRays(128, 96, *scenes.RAYS_1080) == 0
        rt = beam.IRenderTarget.createOffscreen(ctx, 128, 96)
        assert cam.trace(scenes.BUNNY_EYE, scenes.IDENTITY, scene, rt) == beam.ERROR_GPU_ALLOC_FAIL
        assert cam.trace(scenes.BUNNY_EYE, scenes.IDENTITY, scene, rt) == beam.ERROR_NOT_BUILT
        ctx.set_param("kd_max_leaves", -1)
        scene.updateGPUScene()
        assert cam.trace(scenes.BUNNY_EYE, scenes.IDENTITY, scene, rt) == 0
        f = {k: v.reshape(-1) for k, v in rt.read().items()}
        err, rays = oracle.camera_rays(128, 96, *scenes.RAYS_1080)
        packed, tri, t = oracle.kd_render(meshes, rays, scenes.BUNNY_EYE, scenes.IDENTITY)
        assert np.array_equal(f["tri_id"], tri) and np.array_equal(f["packed"], packed) and np.array_equal(f["t"], t)
        assert int(scene.kdStats()[0]) == 16742
        rt.destroy()
        cam.destroy()
        scene.destroy()
        del keep
    finally:
        ctx.close()


@pytest.mark.parametrize("march", [3, 2])
def test_reference_mode_no_grid_records(oracle, march):
    """BM_PARAM_KD_GRID 0 ('never the closed form') now governs the march records too (node,
    leaf and child-box boxes by the halving recurrence); on the grid-exact world the frames are the same."""
    ctx = beam.Context(device=0, reference_kd=True, params={"kd_grid": 0, "kd_march": march})
    try:
        meshes = scenes.load_mesh("bunny")
        err, rays = oracle.camera_rays(160, 120, *scenes.RAYS_1080)
        f, _ = kd_frame(ctx, meshes, 160, 120, scenes.RAYS_1080, scenes.BUNNY_EYE, scenes.IDENTITY)
        packed, tri, t = oracle.kd_render(meshes, rays, scenes.BUNNY_EYE, scenes.IDENTITY)
        assert np.array_equal(f["tri_id"], tri) and np.array_equal(f["packed"], packed) and np.array_equal(f["t"], t)
    finally:
        ctx.close()


@pytest.mark.parametrize("name", ["bunny", "armadillo_proxy", "merged_proxy", "f16"])
def test_reference_mode_ranked_pair_sort(oracle, name):
    """The (leaf, face) pair sort in three passes — the last on the rank of the leaf paths' top 11 bits
    among those the count pass marked (BM_SORT_KD_RANKED, the default) — against the four plain passes
    (BM_PARAM_KD_TOP_RANK 0): the same tree (leaf statistics) and the same frame, equal to the oracle's."""
    meshes = scenes.scene(name)
    eye = (0.0, 0.0, -2.1) if name == "f16" else scenes.BUNNY_EYE
    out = {}
    for rank in (1, 0):
        ctx = beam.Context(device=0, reference_kd=True, params={"kd_top_rank": rank})
        scene = beam.IScene.create(ctx)
        keep = beam.upload_meshes(ctx, scene, meshes)
        st = scene.updateGPUScene(stats=True)
        assert st["sort_path"] == (beam.SORT_KD_RANKED if rank else beam.SORT_LSD), st
        scene.destroy()
        del keep
        out[rank] = kd_frame(ctx, meshes, 320, 180, scenes.RAYS_1080, eye, scenes.IDENTITY)
        ctx.close()
    (f1, s1), (f0, s0) = out[1], out[0]
    assert np.array_equal(s1, s0)
    for k in ("packed", "tri_id", "t"):
        assert np.array_equal(f1[k].view(np.uint32), f0[k].view(np.uint32)), k
    err, rays = oracle.camera_rays(320, 180, *scenes.RAYS_1080)
    packed, tri, t = oracle.kd_render(meshes, rays, eye, scenes.IDENTITY)
    assert np.array_equal(f1["tri_id"], tri) and np.array_equal(f1["packed"], packed)
    assert np.array_equal(f1["t"], t)


def test_reference_mode_ranked_sort_falls_back_when_top_bits_spread(oracle):
    """Triangles scattered over the whole ±30 world: their leaf paths' top 11 bits take more than 1,024
    values, so the pair sort keeps its four plain passes (BM_SORT_LSD) with the ranked digit enabled;
    the frame equals the oracle's."""
    rng = np.random.default_rng(11)
    n = 20000
    c = rng.uniform(-28.0, 28.0, size=(n, 1, 3)).astype(np.float32)
    pos = (c + rng.uniform(-0.6, 0.6, size=(n, 3, 3)).astype(np.float32)).reshape(-1, 3)
    nrm = np.tile(np.array([0.0, 0.0, -1.0], np.float32), (pos.shape[0], 1))
    meshes = [{"pos": pos, "nrm": nrm, "idx": np.arange(pos.shape[0], dtype=np.uint32)}]
    eye = (0.0, 0.0, -29.5)
    ctx = beam.Context(device=0, reference_kd=True)
    scene = beam.IScene.create(ctx)
    keep = beam.upload_meshes(ctx, scene, meshes)
    st = scene.updateGPUScene(stats=True)
    assert st["sort_path"] == beam.SORT_LSD, st
    scene.destroy()
    del keep
    f, _ = kd_frame(ctx, meshes, 128, 128, scenes.RAYS_SQUARE, eye, scenes.IDENTITY)
    ctx.close()
    err, rays = oracle.camera_rays(128, 128, *scenes.RAYS_SQUARE)
    packed, tri, t = oracle.kd_render(meshes, rays, eye, scenes.IDENTITY)
    assert (tri != 0xFFFFFFFF).any()
    assert np.array_equal(f["tri_id"], tri) and np.array_equal(f["packed"], packed)
    assert np.array_equal(f["t"], t)


def test_reference_mode_out_of_range_and_nan_triangles(oracle):
    """The walks test a triangle with coordinates below 2^60 by the min/max form of the triangle/box test
    (tri_box_finite) and any other by the reference's exact sequence: the bunny plus triangles far outside
    the world (products overflow), one reaching from inside the world to 1e19 and one with a NaN vertex,
    so waves run both forms side by side. Tree statistics and frame equal the oracle's."""
    bunny = scenes.load_mesh("bunny")
    pos = np.array([[1e20, 1e20, 1e20], [2e20, 1e20, 1e20], [1e20, 3e20, -1e20],
                    [0.1, 0.1, 0.1], [0.1001, 0.1, 0.1], [1e19, 1e19, 5.0],
                    [0.2, 0.2, 0.2], [np.nan, 0.3, 0.2], [0.2, 0.4, 0.2]], np.float32)
    nrm = np.tile(np.array([0.0, 0.0, -1.0], np.float32), (pos.shape[0], 1))
    meshes = list(bunny) + [{"pos": pos, "nrm": nrm, "idx": np.arange(9, dtype=np.uint32)}]
    ctx = beam.Context(device=0, reference_kd=True)
    try:
        err, rays = oracle.camera_rays(160, 120, *scenes.RAYS_1080)
        f, st = kd_frame(ctx, meshes, 160, 120, scenes.RAYS_1080, scenes.BUNNY_EYE, scenes.IDENTITY)
        packed, tri, t, ost = oracle.kd_render(meshes, rays, scenes.BUNNY_EYE, scenes.IDENTITY, stats=True)
        assert (tri != 0xFFFFFFFF).any()
        assert np.array_equal(f["tri_id"], tri) and np.array_equal(f["packed"], packed)
        assert np.array_equal(f["t"], t)
        assert int(st[1]) == int(ost[2]) and int(st[2]) == int(ost[3])
    finally:
        ctx.close()
