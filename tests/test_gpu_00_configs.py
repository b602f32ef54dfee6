"""BASELINE.json configs end to end on the GPU, collected before every other GPU test (file name) so
that no earlier stop under `pytest -x` can hide them.

  C1  bunny / suzanne / f16 golden views (the reference's frames, tests/golden/views)
  C2  bunny 1920x1080, every pixel (+ the SURVEY §8(c) known answer)
  C3  armadillo proxy 1920x1080 vs the oracle
  C4  armadillo proxy 3840x2160, whole frame + the 2/4/8-way band shares reassembled
  C5  tyra+f16 merged proxy (1,118,136 tris) 1920x1080 + one shadow ray per hit
  ref reference mode (the reference's kd-tree and first-hit-leaf march): golden frames on every pixel

Bars (BASELINE.json north_star): triangle ids and packed colours bit-exact; t and rgb within 1e-5 (t is
bit-exact: same operations, no contraction). Against the reference frames the only allowed
differences in closest-hit mode are the recorded early-out pixels, where the reference's
first-hit-leaf exit (BuildTree.cu:427-431) returns a farther triangle than the closest hit; reference
mode has none.
"""
import numpy as np
import pytest

from golden_io import closest_hit_expected, dense, manifest, view
from gpu_util import assert_frame_equal, gpu_build, gpu_frame, kd_frame, oracle_frame, oracle_shadow, shadow_frame
from raytracercuda_amd import beam, multigpu, scenes

pytestmark = pytest.mark.gpu

C5_LIGHT = (0.0, 10.0, -10.0)
RAYS_4K = (-16.0 / 9.0, 16.0 / 9.0, -1.0, 1.0, 1.0)


@pytest.fixture(scope="module")
def kctx():
    c = beam.Context(device=0, reference_kd=True)
    yield c
    c.close()


@pytest.mark.parametrize("name", ["bunny_256", "suzanne_256", "f16_500"])
def test_c1_golden_views(ctx, oracle, name):
    m = manifest()["views"][name]
    meshes = scenes.load_mesh(m["mesh"])
    scene, keep, _ = gpu_build(ctx, meshes)
    f = gpu_frame(ctx, scene, m["w"], m["h"], m["rays"], m["eye"], scenes.IDENTITY, rgb=True)
    # 1) the closest-hit oracle, every pixel
    assert_frame_equal(f, *oracle_frame(oracle, meshes, m["w"], m["h"], m["rays"], m["eye"], scenes.IDENTITY))
    # 2) the reference frame: identical except the recorded early-out pixels
    g = view(name)
    rp, rt_, rtt = dense(m["w"] * m["h"], g)
    diff = np.nonzero(f["tri_id"] != rt_)[0]
    assert np.array_equal(diff, g["div_pixels"])
    same = np.ones(rp.size, bool)
    same[g["div_pixels"]] = False
    assert np.array_equal(f["packed"][same], rp[same])
    assert np.array_equal(f["t"][same], rtt[same])
    # 3) shaded rgb: (|n.z|, 0, 0) on a hit, (0, 1, 0) on a miss, consistent with packed
    hit = f["tri_id"] != 0xFFFFFFFF
    rgb = f["rgb"]
    assert np.all(rgb[~hit] == np.array([0, 1, 0], np.float32))
    assert np.all(rgb[hit, 1:] == 0)
    red = (f["packed"][hit] >> 16).astype(np.float32)
    assert np.all(np.floor(rgb[hit, 0] * np.float32(255)) == red)
    scene.destroy()


def test_c2_bunny_1080_every_pixel(ctx):
    m = manifest()["views"]["bunny_1080"]
    meshes = scenes.load_mesh("bunny")
    scene, keep, _ = gpu_build(ctx, meshes)
    f = gpu_frame(ctx, scene, m["w"], m["h"], m["rays"], m["eye"], scenes.IDENTITY)
    n = m["w"] * m["h"]
    assert_frame_equal(f, *closest_hit_expected(n, view("bunny_1080")))
    hits = int((f["tri_id"] != 0xFFFFFFFF).sum())
    assert hits == m["closest_hit_hits"]
    assert int(f["packed"].astype(np.uint64).sum()) == m["closest_hit_checksum"]
    # reference checksum once the 3 early-out pixels take the reference's answer
    g = view("bunny_1080")
    p = f["packed"].copy()
    rp, _, _ = dense(n, g)
    p[g["div_pixels"]] = rp[g["div_pixels"]]
    assert int(p.astype(np.uint64).sum()) == m["survey_known_answer"]["checksum"]
    scene.destroy()


def test_c3_armadillo_proxy_1080(ctx, oracle):
    meshes = scenes.scene("armadillo_proxy")
    scene, keep, st = gpu_build(ctx, meshes)
    assert st["num_tris"] == 278520
    f = gpu_frame(ctx, scene, 1920, 1080, scenes.RAYS_1080, scenes.BUNNY_EYE, scenes.IDENTITY)
    assert_frame_equal(f, *oracle_frame(oracle, meshes, 1920, 1080, scenes.RAYS_1080, scenes.BUNNY_EYE,
                                        scenes.IDENTITY))
    scene.destroy()


def test_c4_armadillo_4k_full_frame_and_bands(ctx, oracle):
    """Armadillo proxy at 3840x2160: the whole frame equals the oracle's bit for bit, and the
    2/4/8-way band shares (what each GPU traces before the gather) reassemble into it."""
    meshes = scenes.scene("armadillo_proxy")
    scene, keep, st = gpu_build(ctx, meshes)
    w, h, bh = 3840, 2160, 16
    f = gpu_frame(ctx, scene, w, h, RAYS_4K, scenes.BUNNY_EYE, scenes.IDENTITY)
    assert_frame_equal(f, *oracle_frame(oracle, meshes, w, h, RAYS_4K, scenes.BUNNY_EYE, scenes.IDENTITY))
    cam = beam.ICamera.create(ctx)
    assert cam.setInitialRays(w, h, *RAYS_4K) == 0
    for world in (2, 4, 8):
        rows = multigpu.rows_per_rank(h, bh, world)
        parts = []
        for r in range(world):
            rt = beam.IRenderTarget.createOffscreen(ctx, w, rows)
            assert cam.traceBands(scenes.BUNNY_EYE, scenes.IDENTITY, scene, rt, bh, world, r) == 0
            got = rt.read()
            parts.append(np.stack([got["packed"], got["tri_id"], got["t"].view(np.uint32)]))
            rt.destroy()
        frame = multigpu.reassemble_np(np.stack(parts), h, bh)
        assert np.array_equal(frame[0].reshape(-1), f["packed"])
        assert np.array_equal(frame[1].reshape(-1), f["tri_id"])
        assert np.array_equal(frame[2].reshape(-1), f["t"].view(np.uint32))
    cam.destroy()
    scene.destroy()


def test_c5_merged_proxy_1080_with_shadows(ctx, oracle):
    """tyra+f16 proxy (1,118,136 tris, 3 meshes) at 1920x1080, light (0,10,-10)."""
    meshes = scenes.scene("merged_proxy")
    scene, keep, _ = gpu_build(ctx, meshes)
    f, cnt = shadow_frame(ctx, scene, 1920, 1080, scenes.RAYS_1080, scenes.BUNNY_EYE, scenes.IDENTITY, C5_LIGHT,
                          counters=True)
    packed, tri, t, sh, ocnt = oracle_shadow(oracle, meshes, 1920, 1080, scenes.RAYS_1080, scenes.BUNNY_EYE,
                                             scenes.IDENTITY, C5_LIGHT)
    assert np.array_equal(f["tri_id"], tri)
    assert np.array_equal(f["packed"], packed)
    assert np.array_equal(f["t"], t)
    assert np.array_equal(f["shadow"], sh), f"{int((f['shadow'] != sh).sum())} shadow pixels differ"
    assert int(sh.sum()) > 0
    assert list(map(int, cnt[3:])) == list(map(int, ocnt))
    scene.destroy()


@pytest.mark.parametrize("name", ["bunny_256", "suzanne_256", "f16_500", "bunny_1080"])
def test_reference_mode_golden_frames_every_pixel(kctx, oracle, name):
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


def test_c4_multi_device_context_2_4_8(ctx):
    """C4 through the C ABI's multi-device context (bm_options.devices): the armadillo proxy at
    3840x2160 with 16-row bands dealt over 2/4/8 band devices (all on this one GPU: the rehearsal of
    the 8-GPU path) and gathered into the root's render target by the peer-write kernel equals the
    single-device frame (itself equal to the oracle above) on every plane."""
    meshes = scenes.scene("armadillo_proxy")
    scene, keep, _ = gpu_build(ctx, meshes)
    ref = gpu_frame(ctx, scene, 3840, 2160, RAYS_4K, scenes.BUNNY_EYE, scenes.IDENTITY, rgb=True)
    scene.destroy()
    del keep
    for n in (2, 4, 8):
        mctx = beam.Context(device=0, devices=[0] * n)
        assert mctx.num_devices == n
        ms, mkeep, _ = gpu_build(mctx, meshes)
        f = gpu_frame(mctx, ms, 3840, 2160, RAYS_4K, scenes.BUNNY_EYE, scenes.IDENTITY, rgb=True)
        for k in ("packed", "tri_id", "t", "rgb"):
            assert np.array_equal(f[k], ref[k]), f"{n} devices: plane {k} differs"
        ms.destroy()
        del mkeep
        mctx.close()


def test_filled_view_armadillo_proxy_1080(ctx, oracle):
    """The bench's filled-view side figure (armadillo proxy, eye close: 85.5 % of pixels hit) vs the
    oracle on every pixel."""
    c = scenes.CONFIGS["filled"]
    meshes = scenes.scene(c["scene"])
    scene, keep, _ = gpu_build(ctx, meshes)
    f = gpu_frame(ctx, scene, c["width"], c["height"], c["rays"], c["eye"], scenes.IDENTITY)
    exp = oracle_frame(oracle, meshes, c["width"], c["height"], c["rays"], c["eye"], scenes.IDENTITY)
    assert_frame_equal(f, *exp)
    assert (exp[1] != 0xFFFFFFFF).mean() > 0.8
    scene.destroy()


@pytest.mark.parametrize("cfg,want", [("filled", "packets"), ("c4", "packets"), ("c3", "quads"), ("c2", "quads")])
def test_auto_kernel_choice(oracle, cfg, want):
    """The default context picks wave packets (k_trace_packet) for dense coherent views — the scene box
    covering >= 1M of the target's pixels at >= 4 pixels per triangle — and ray quads otherwise; with
    BM_PARAM_TRACE_AUTO_PACKET 0 it keeps quads. The two frames are bit-identical, and the filled view's ids
    equal the oracle's (the C4 test above compares the whole default-context 4K frame with the oracle)."""
    c = scenes.CONFIGS[cfg]
    meshes = scenes.scene(c["scene"])
    kinds = {}
    frames = {}
    for auto in (1, 0):
        ctx = beam.Context(device=0, params={"trace_auto_packet": auto})
        scene, keep, _ = gpu_build(ctx, meshes)
        cam = beam.ICamera.create(ctx)
        assert cam.setInitialRays(c["width"], c["height"], *c["rays"]) == 0
        rt = beam.IRenderTarget.createOffscreen(ctx, c["width"], c["height"])
        assert cam.trace(c["eye"], scenes.IDENTITY, scene, rt) == 0
        kinds[auto] = rt.traceKind()
        frames[auto] = rt.read()
        rt.destroy()
        cam.destroy()
        scene.destroy()
        del keep
        ctx.close()
    assert kinds[1] == want and kinds[0] == "quads"
    for k in ("packed", "tri_id", "t"):
        assert np.array_equal(frames[1][k].view(np.uint32), frames[0][k].view(np.uint32)), k
    if cfg == "filled":
        exp = oracle_frame(oracle, meshes, c["width"], c["height"], c["rays"], c["eye"], scenes.IDENTITY)
        assert np.array_equal(frames[1]["tri_id"].reshape(-1), exp[1])


@pytest.mark.parametrize("cfg,want", [("filled", "packets"), ("c2", "packets"), ("c3", "cull+quads")])
def test_packets_frames_in_flight(oracle, cfg, want):
    """Frames in flight: three render targets on their own HIP streams, two rounds back to back, with the
    kernel the default context picks for them (wave packets down to 0.5M covered pixels: the filled view
    and the bunny at 1080p; the compacted quads for C3); every frame equals the oracle's (ids, packed
    colours, t bits)."""
    import torch
    c = scenes.CONFIGS[cfg]
    meshes = scenes.scene(c["scene"])
    exp = oracle_frame(oracle, meshes, c["width"], c["height"], c["rays"], c["eye"], scenes.IDENTITY)
    ctx = beam.Context(device=0)
    scene, keep, _ = gpu_build(ctx, meshes)
    cam = beam.ICamera.create(ctx)
    assert cam.setInitialRays(c["width"], c["height"], *c["rays"]) == 0
    streams = [torch.cuda.Stream(device=0) for _ in range(3)]
    rts = [beam.IRenderTarget.createOffscreen(ctx, c["width"], c["height"]) for _ in range(3)]
    for rt, st in zip(rts, streams):
        rt.setStream(st.cuda_stream)
    for _ in range(2):
        for rt in rts:
            assert cam.trace(c["eye"], scenes.IDENTITY, scene, rt) == 0
        for rt in rts:
            assert rt.traceKind() == want
            f = {k: v.reshape(-1) for k, v in rt.read().items()}
            assert_frame_equal(f, *exp)
    for rt in rts:
        rt.destroy()
    cam.destroy()
    scene.destroy()
    del keep
    ctx.close()
