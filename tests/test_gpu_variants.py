"""GPU parity of every trace kernel the library can select (bm_internal.h TraceVariant): the single-
lane persistent kernel (8x8 pixels per wave), the ray-quad kernel (four lanes per ray, 4x4 pixels
per wave; block-dynamic and cost-ordered tile order) and the compacted quad kernel (lane-per-ray
setup and root cull, LDS ray queue, quads for the survivors); in an A/B build also the static tile
orders, the quad kernel with in-wave ray refill and the ray-pair kernel. Each must
give the oracle's frame (ids, packed colours, t bit-exact), its traversal counters and, with shadow
rays, its shadow plane and shadow counters — on full frames, ragged frames, bands, leaf sizes 1/4/16
and BVH2 scenes (which the quad variants hand to the single-lane kernel).

The variant and tile order are tuning parameters of a context (bm_context_set_param:
BM_PARAM_TRACE_VARIANT / BM_PARAM_TRACE_SCHED); the library reads nothing from the environment."""
import numpy as np
import pytest

from raytracercuda_amd import beam, scenes

pytestmark = pytest.mark.gpu

PRIO12, QUAD, QUAD_FETCH, COMPACT, PAIR, PACKET = 6, 10, 11, 12, 13, 14
# the product kernels (every path the in-tree library can take) ...
VARIANTS = [(PRIO12, None), (QUAD, "1"), (QUAD, "2"), (COMPACT, "1"), (PACKET, None)]
IDS = ["single-lane", "quad-dynamic", "quad-costorder", "compact-dynamic", "packet"]
# (wave packets trace non-counting BVH4 primary frames; counting and shadow traces of that variant run the
# quad kernel, so each test below checks the packet frame against the oracle and the quad counters)
# ... and, in an A/B build (BEAM_HIP_LIB=<tools/build_ab.py ... BM_TRACE_AB=1 output>), the variants
# measured slower (bm_trace_ab.hip) and the static tile orders
if beam.ab_build():
    VARIANTS += [(QUAD, "0"), (QUAD_FETCH, None), (COMPACT, "0"), (PAIR, None)]
    IDS += ["quad-static", "quad-refill", "compact-static", "pair"]
LIGHT = (0.0, 10.0, -10.0)


@pytest.fixture(params=VARIANTS, ids=IDS)
def vctx(request):
    variant, sched = request.param
    params = {"trace_variant": variant}
    if sched is not None:
        params["trace_sched"] = int(sched)
    made = []

    def make(**kw):
        c = beam.Context(device=0, params=params, **kw)
        made.append(c)
        return c

    yield make
    for c in made:
        c.close()


def render(ctx, meshes, w, h, cam, eye, orient, light=None):
    scene = beam.IScene.create(ctx)
    keep = beam.upload_meshes(ctx, scene, meshes)
    scene.updateGPUScene()
    c = beam.ICamera.create(ctx)
    assert c.setInitialRays(w, h, *cam) == 0
    rt = beam.IRenderTarget.createOffscreen(ctx, w, h)
    if light is None:
        cnt = c.traceCounters(eye, orient, scene, rt)
        assert c.trace(eye, orient, scene, rt) == 0
    else:
        cnt = c.traceShadowCounters(eye, orient, scene, rt, light)
        assert c.traceShadow(eye, orient, scene, rt, light) == 0
    f = {k: v.reshape(-1) for k, v in rt.read().items()}
    if light is not None:
        f["shadow"] = rt.readShadow().reshape(-1)
    rt.destroy()
    c.destroy()
    scene.destroy()
    del keep
    return f, cnt


def expect(oracle, meshes, w, h, cam, eye, orient, leaf=4, width=4, light=None):
    err, rays = oracle.camera_rays(w, h, *cam)
    assert err == 0
    bvh = oracle.bvh_build(meshes, leaf, width)
    packed, tri, t, cnt = bvh.render(rays, eye, orient, counters=True)
    out = {"packed": packed, "tri_id": tri, "t": t}
    if light is not None:
        sh, scnt = bvh.shadow(rays, eye, orient, light, tri, t, counters=True)
        out["shadow"] = sh
        cnt = np.concatenate([cnt, scnt])
    return out, cnt


def check(f, cnt, exp, ecnt):
    for k, v in exp.items():
        got = f[k].view(np.uint32) if f[k].dtype == np.float32 else f[k]
        want = v.view(np.uint32) if v.dtype == np.float32 else v
        assert np.array_equal(got, want), f"{k}: {int((got != want).sum())} pixels differ"
    assert list(cnt) == list(ecnt)


@pytest.mark.parametrize("name,leaf", [("bunny", 4), ("suzanne", 1), ("f16", 16), ("armadillo_proxy", 4)])
def test_variant_frames_and_counters(vctx, oracle, name, leaf):
    ctx = vctx(leaf_size=leaf)
    meshes = scenes.scene(name)
    w, h = (480, 270) if name != "armadillo_proxy" else (1920, 1080)
    eye = scenes.BUNNY_EYE if name in ("bunny", "armadillo_proxy") else (0.0, 0.0, -3.0)
    f, cnt = render(ctx, meshes, w, h, scenes.RAYS_1080, eye, scenes.IDENTITY)
    check(f, cnt, *expect(oracle, meshes, w, h, scenes.RAYS_1080, eye, scenes.IDENTITY, leaf))


def test_variant_bvh2_fallback(vctx, oracle):
    ctx = vctx(bvh_width=2)
    meshes = scenes.scene("bunny")
    f, cnt = render(ctx, meshes, 320, 180, scenes.RAYS_1080, scenes.BUNNY_EYE, scenes.IDENTITY)
    check(f, cnt, *expect(oracle, meshes, 320, 180, scenes.RAYS_1080, scenes.BUNNY_EYE, scenes.IDENTITY, width=2))


@pytest.mark.parametrize("w,h", [(1, 1), (5, 3), (37, 23), (130, 67)])
def test_variant_ragged_frames(vctx, oracle, w, h):
    ctx = vctx()
    rng = np.random.default_rng(w * 131 + h)
    n = 40
    meshes = [{"pos": rng.uniform(-1, 1, size=(3 * n, 3)).astype(np.float32),
               "nrm": rng.normal(size=(3 * n, 3)).astype(np.float32), "idx": np.arange(3 * n, dtype=np.uint32)}]
    f, cnt = render(ctx, meshes, w, h, scenes.RAYS_SQUARE, (0.1, 0.05, -3), scenes.IDENTITY)
    check(f, cnt, *expect(oracle, meshes, w, h, scenes.RAYS_SQUARE, (0.1, 0.05, -3), scenes.IDENTITY))


def test_variant_sweep_views(vctx, oracle):
    ctx = vctx()
    meshes = scenes.scene("bunny")
    rng = np.random.default_rng(7)
    for _ in range(3):
        d = rng.normal(size=3)
        d /= np.linalg.norm(d)
        eye = (np.array([-0.337, 1.203, -0.031]) + 3.0 * d).astype(np.float32)
        fwd = -d
        right = np.cross([0, 1, 0], fwd)
        right /= np.linalg.norm(right)
        up = np.cross(fwd, right)
        orient = np.stack([right, up, fwd], 1).astype(np.float32).T.reshape(-1)  # column-major mat3
        f, cnt = render(ctx, meshes, 256, 144, scenes.RAYS_1080, tuple(eye), orient)
        check(f, cnt, *expect(oracle, meshes, 256, 144, scenes.RAYS_1080, tuple(eye), orient))


@pytest.mark.parametrize("orient", [
    (1.3, 0.2, 0.0, 0.0, 0.9, 0.1, 0.05, 0.0, 1.1),     # sheared and scaled: exact ray setup in the cull
    (0.0, 1.0, 0.0, -1.0, 0.0, 0.0, 0.0, 0.0, 1.0),     # a 90-degree roll: axis-exact directions
    (1.0, 0.0, 0.0, 0.0, 1.0, 0.0, 0.0, 0.0, -1.0)])    # mirrored: looking away from the bunny
def test_variant_general_orient(vctx, oracle, orient):
    """Non-rotation and axis-aligned orient matrices (the compacted variant's root cull picks its
    exact or approximate ray setup from the orient; zero direction components reach the slab
    tests as infinite reciprocals)."""
    ctx = vctx()
    meshes = scenes.scene("bunny")
    o = np.asarray(orient, np.float32)
    f, cnt = render(ctx, meshes, 320, 180, scenes.RAYS_1080, scenes.BUNNY_EYE, o)
    check(f, cnt, *expect(oracle, meshes, 320, 180, scenes.RAYS_1080, scenes.BUNNY_EYE, o))


@pytest.mark.parametrize("name", ["bunny", "f16"])
def test_variant_shadow(vctx, oracle, name):
    ctx = vctx()
    meshes = scenes.scene(name)
    eye = scenes.BUNNY_EYE if name == "bunny" else (0.0, 0.0, -3.0)
    f, cnt = render(ctx, meshes, 400, 225, scenes.RAYS_1080, eye, scenes.IDENTITY, light=LIGHT)
    check(f, cnt, *expect(oracle, meshes, 400, 225, scenes.RAYS_1080, eye, scenes.IDENTITY, light=LIGHT))


def test_variant_bands(vctx):
    ctx = vctx()
    meshes = scenes.scene("bunny")
    scene = beam.IScene.create(ctx)
    keep = beam.upload_meshes(ctx, scene, meshes)
    scene.updateGPUScene()
    w, h, bh, n = 300, 170, 16, 3
    cam = beam.ICamera.create(ctx)
    assert cam.setInitialRays(w, h, *scenes.RAYS_1080) == 0
    full_rt = beam.IRenderTarget.createOffscreen(ctx, w, h)
    assert cam.trace(scenes.BUNNY_EYE, scenes.IDENTITY, scene, full_rt) == 0
    full = full_rt.read()
    for r in range(n):
        bands = (h + bh - 1) // bh
        mine = [b for b in range(bands) if b % n == r]
        rt = beam.IRenderTarget.createOffscreen(ctx, w, len(mine) * bh)
        assert cam.traceBands(scenes.BUNNY_EYE, scenes.IDENTITY, scene, rt, bh, n, r) == 0
        part = rt.read()
        for i, b in enumerate(mine):
            rows = slice(b * bh, min((b + 1) * bh, h))
            k = rows.stop - rows.start
            for plane in ("packed", "tri_id"):
                assert np.array_equal(part[plane][i * bh:i * bh + k], full[plane][rows])
        rt.destroy()
    full_rt.destroy()
    cam.destroy()
    scene.destroy()
    del keep


@pytest.mark.skipif(beam.ab_build(), reason="an A/B build carries BVH8 and every variant")
def test_product_build_refuses_ab_only_options(monkeypatch, oracle):
    """The in-tree library carries the product kernels only: BVH8 and an A/B-only variant are refused
    with BM_ERROR_INVALID_PARAMETER, and stray BM_* variables in the environment change nothing:
    the library reads no environment (ADVICE/VERDICT r3), so the frame and the kernel kind stay the
    default's."""
    with pytest.raises(beam.BeamError) as ei:
        beam.Context(device=0, bvh_width=8)
    assert ei.value.code == beam.ERROR_INVALID_PARAMETER
    with pytest.raises(beam.BeamError) as ei:
        beam.Context(device=0, params={"trace_variant": PAIR})
    assert ei.value.code == beam.ERROR_INVALID_PARAMETER
    for k, v in {"BM_TRACE_VARIANT": str(PRIO12), "BM_TRACE_SCHED": "0", "BM_BVH_WIDTH": "2", "BM_TRACE_GRID": "3",
                 "BM_MSD_MAX_N": "0", "BM_KD_VARIANT": "0"}.items():
        monkeypatch.setenv(k, v)
    ctx = beam.Context(device=0)
    assert all(ctx.get_param(k) == -1 for k in ("trace_variant", "trace_sched", "trace_grid", "msd_max_n"))
    meshes = scenes.scene("bunny")
    f, cnt = render(ctx, meshes, 320, 180, scenes.RAYS_1080, scenes.BUNNY_EYE, scenes.IDENTITY)
    check(f, cnt, *expect(oracle, meshes, 320, 180, scenes.RAYS_1080, scenes.BUNNY_EYE, scenes.IDENTITY))
    sc = beam.IScene.create(ctx)
    keep = beam.upload_meshes(ctx, sc, meshes)
    st = sc.updateGPUScene(stats=True)  # BM_MSD_MAX_N / BM_BVH_WIDTH above are ignored
    assert st["sort_path"] == beam.SORT_MSD and st["bvh_width"] == 4
    sc.destroy()
    del keep
    ctx.close()
