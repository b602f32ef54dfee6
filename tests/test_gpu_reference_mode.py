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

from golden_io import dense, manifest, view
from raytracercuda_amd import beam, scenes

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def kctx():
    c = beam.Context(device=0, reference_kd=True)
    yield c
    c.close()


def kd_frame(ctx, meshes, w, h, cam, eye, orient):
    scene = beam.IScene.create(ctx)
    keep = beam.upload_meshes(ctx, scene, meshes)
    scene.updateGPUScene(stats=True)
    c = beam.ICamera.create(ctx)
    assert c.setInitialRays(w, h, *cam) == 0
    rt = beam.IRenderTarget.createOffscreen(ctx, w, h)
    assert c.trace(eye, orient, scene, rt) == 0
    f = {k: v.reshape(-1) for k, v in rt.read().items()}
    stats = scene.kdStats()
    rt.destroy()
    c.destroy()
    scene.destroy()
    del keep
    return f, stats


@pytest.mark.parametrize("name", ["bunny_256", "suzanne_256", "f16_500", "bunny_1080"])
def test_reference_frames_bit_exact_on_every_pixel(kctx, oracle, name):
    m = manifest()["views"][name]
    meshes = scenes.load_mesh(m["mesh"])
    f, st = kd_frame(kctx, meshes, m["w"], m["h"], m["rays"], m["eye"], scenes.IDENTITY)
    packed, tri, t = dense(m["w"] * m["h"], view(name))
    assert np.array_equal(f["tri_id"], tri), f"{int((f['tri_id'] != tri).sum())} ids differ"
    assert np.array_equal(f["packed"], packed)
    assert np.array_equal(f["t"], t)
    # the SURVEY known answer itself: hits and the sum of the packed framebuffer
    kh = m["survey_known_answer"]
    assert int((packed != 0xFF00).sum()) == kh["hits"] == int((f["packed"] != 0xFF00).sum())
    assert int(f["packed"].astype(np.uint64).sum()) == kh["checksum"]
    # the early-out pixels are where this mode differs from the closest-hit modes
    assert np.array_equal(f["tri_id"][view(name)["div_pixels"]], tri[view(name)["div_pixels"]])
    ost = oracle.kd_render(meshes, np.zeros((1, 3), np.float32), m["eye"], scenes.IDENTITY, stats=True)[3]
    assert [int(st[1]), int(st[2])] == [int(ost[2]), int(ost[3])]  # face refs stored, dropped
    assert int(min(st[3], 256)) == int(min(ost[4], 256))


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
