"""Hashed-grid mode (BM_OPT_REFERENCE_HASH): the reference's alternative accelerator (Raytracer/Hash.cu,
SURVEY §8(f) 4) built and marched on the GPU.

Bar: the buckets (start, end, face order) equal the oracle's restatement, and every pixel's packed
colour, triangle id and t equals the oracle's march bit for bit (oracle/beam_oracle.c orc_hash_*).
Parity with the reference itself is unpinned: it never shipped this configuration (Types.h:13)."""
import numpy as np
import pytest

from raytracercuda_amd import beam, scenes

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def hctx():
    c = beam.Context(device=0, reference_hash=True)
    yield c
    c.close()


def hash_frame(ctx, meshes, w, h, cam, eye, orient, export=False):
    scene = beam.IScene.create(ctx)
    keep = beam.upload_meshes(ctx, scene, meshes)
    scene.updateGPUScene(stats=True)
    c = beam.ICamera.create(ctx)
    assert c.setInitialRays(w, h, *cam) == 0
    rt = beam.IRenderTarget.createOffscreen(ctx, w, h)
    assert c.trace(eye, orient, scene, rt) == 0
    f = {k: v.reshape(-1) for k, v in rt.read().items()}
    stats = scene.gridStats()
    ex = scene.gridExport() if export else None
    rt.destroy()
    c.destroy()
    scene.destroy()
    del keep
    return f, stats, ex


def check(oracle, ctx, meshes, w, h, cam, eye, orient, export=False):
    f, st, ex = hash_frame(ctx, meshes, w, h, cam, eye, orient, export)
    err, rays = oracle.camera_rays(w, h, *cam)
    assert err == 0
    res = oracle.hash_render(meshes, rays, eye, orient, stats=True, buckets=export)
    packed, tri, t, ost = res[:4]
    assert list(st) == [int(x) for x in ost]
    assert np.array_equal(f["tri_id"], tri), f"{int((f['tri_id'] != tri).sum())} ids differ"
    assert np.array_equal(f["packed"], packed)
    assert np.array_equal(f["t"].view(np.uint32), t.view(np.uint32))
    if export:
        start, faces = res[4]
        b0, b1, gf = ex
        assert np.array_equal(b0[b1 > b0], start[:-1][b1 > b0])
        assert np.array_equal(b1 - b0, np.diff(start))
        assert np.array_equal(gf, faces)
    return f, st


@pytest.mark.parametrize("name,w,eye", [("bunny", 96, scenes.BUNNY_EYE), ("f16", 128, (0.0, 0.0, -2.1)),
                                        ("suzanne", 128, (0.0, 0.0, -3.0))])
def test_hash_frames_and_buckets(hctx, oracle, name, w, eye):
    f, st = check(oracle, hctx, scenes.scene(name), w, w, scenes.RAYS_SQUARE, eye, scenes.IDENTITY, export=True)
    assert (f["tri_id"] != 0xFFFFFFFF).any()


def test_hash_general_view(hctx, oracle):
    o = np.float32([0.0, 1.0, 0.0, -1.0, 0.0, 0.0, 0.0, 0.0, 1.0])  # rolled 90 degrees: zero direction parts
    check(oracle, hctx, scenes.scene("f16"), 64, 48, scenes.RAYS_1080, (0.05, -0.02, -2.1), o)


def test_hash_tiny_scenes(hctx, oracle):
    rng = np.random.default_rng(5)
    for n in (1, 2, 17):
        pos = rng.uniform(-0.3, 0.3, size=(3 * n, 3)).astype(np.float32)
        m = [{"pos": pos, "nrm": rng.normal(size=(3 * n, 3)).astype(np.float32),
              "idx": np.arange(3 * n, dtype=np.uint32)}]
        check(oracle, hctx, m, 37, 23, scenes.RAYS_SQUARE, (0.01, 0.02, -1.5), scenes.IDENTITY, export=True)


def test_hash_empty_scene(hctx):
    scene = beam.IScene.create(hctx)
    scene.updateGPUScene()
    c = beam.ICamera.create(hctx)
    assert c.setInitialRays(8, 8, *scenes.RAYS_SQUARE) == 0
    rt = beam.IRenderTarget.createOffscreen(hctx, 8, 8)
    assert c.trace((0, 0, -3), scenes.IDENTITY, scene, rt) == 0
    f = rt.read()
    assert np.all(f["packed"] == 0xFF00) and np.all(f["tri_id"] == 0xFFFFFFFF)
    assert list(scene.gridStats()) == [0, 0, 0, 0]
    rt.destroy()
    c.destroy()
    scene.destroy()


def test_hash_limits_and_errors(hctx):
    # a triangle spanning more than 2^20 cells is refused at build time
    big = [{"pos": np.float32([[-20, -20, 0], [20, -20, 0], [-20, 20, 0.5]]),
            "nrm": np.float32([[0, 0, -1]] * 3), "idx": np.arange(3, dtype=np.uint32)}]
    scene = beam.IScene.create(hctx)
    keep = beam.upload_meshes(hctx, scene, big)
    with pytest.raises(beam.BeamError):
        scene.updateGPUScene()
    scene.destroy()
    del keep
    # only full-frame primary traces: bands, shadows and counters are refused
    scene = beam.IScene.create(hctx)
    keep = beam.upload_meshes(hctx, scene, scenes.scene("f16"))
    scene.updateGPUScene()
    c = beam.ICamera.create(hctx)
    assert c.setInitialRays(32, 32, *scenes.RAYS_SQUARE) == 0
    rt = beam.IRenderTarget.createOffscreen(hctx, 32, 32)
    assert c.traceShadow((0, 0, -2.1), scenes.IDENTITY, scene, rt, (0.0, 10.0, -10.0)) != 0
    assert c.traceBands((0, 0, -2.1), scenes.IDENTITY, scene, rt, 16, 2, 0) != 0
    with pytest.raises(beam.BeamError):
        scene.export()
    rt.destroy()
    c.destroy()
    scene.destroy()
    del keep


def test_hash_and_kd_exclusive():
    with pytest.raises(beam.BeamError):
        beam.Context(device=0, reference_kd=True, reference_hash=True)
