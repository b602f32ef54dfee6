"""Shared helpers of the GPU parity tests: build, trace and read back through the C ABI, and the
oracle frames they are compared with (test infrastructure only)."""
import numpy as np

from raytracercuda_amd import beam

T_TOL = 1e-5  # BASELINE north_star: FP32 t within 1e-5 (it is bit-exact in practice: same op order)


def gpu_build(ctx, meshes):
    scene = beam.IScene.create(ctx)
    keep = beam.upload_meshes(ctx, scene, meshes)
    stats = scene.updateGPUScene(stats=True)
    return scene, keep, stats


def gpu_frame(ctx, scene, w, h, cam, eye, orient, pitch=0, rgb=False):
    c = beam.ICamera.create(ctx)
    assert c.setInitialRays(w, h, *cam) == 0
    rt = beam.IRenderTarget.createOffscreen(ctx, w, h, pitch)
    assert c.trace(eye, orient, scene, rt) == 0
    f = rt.read(rgb=rgb)
    rt.destroy()
    c.destroy()
    return {k: v.reshape(-1) if k != "rgb" else v.reshape(-1, 3) for k, v in f.items()}


def oracle_frame(oracle, meshes, w, h, cam, eye, orient, leaf=4):
    err, rays = oracle.camera_rays(w, h, *cam)
    assert err == 0
    return oracle.bvh_build(meshes, leaf).render(rays, eye, orient)


def assert_frame_equal(f, packed, tri, t):
    assert np.array_equal(f["tri_id"], tri), f"tri mismatches: {int((f['tri_id'] != tri).sum())}"
    assert np.array_equal(f["packed"], packed), f"packed mismatches: {int((f['packed'] != packed).sum())}"
    hit = tri != 0xFFFFFFFF
    assert np.all(np.isinf(f["t"][~hit]))
    assert np.allclose(f["t"][hit], t[hit], rtol=0, atol=T_TOL)
    assert np.array_equal(f["t"], t)  # bit-exact in practice


def shadow_frame(ctx, scene, w, h, cam, eye, orient, light, counters=False):
    c = beam.ICamera.create(ctx)
    assert c.setInitialRays(w, h, *cam) == 0
    rt = beam.IRenderTarget.createOffscreen(ctx, w, h)
    if counters:
        cnt = c.traceShadowCounters(eye, orient, scene, rt, light)
    else:
        assert c.traceShadow(eye, orient, scene, rt, light) == 0
        cnt = None
    f = {k: v.reshape(-1) for k, v in rt.read().items()}
    f["shadow"] = rt.readShadow().reshape(-1)
    rt.destroy()
    c.destroy()
    return f, cnt


def oracle_shadow(oracle, meshes, w, h, cam, eye, orient, light, width=4):
    err, rays = oracle.camera_rays(w, h, *cam)
    assert err == 0
    bvh = oracle.bvh_build(meshes, 4, width)
    packed, tri, t = bvh.render(rays, eye, orient)
    sh, cnt = bvh.shadow(rays, eye, orient, light, tri, t, counters=True)
    return packed, tri, t, sh, cnt


def kd_frame(ctx, meshes, w, h, cam, eye, orient):
    """Reference mode (BM_OPT_REFERENCE_KD context): build, trace, read, kd statistics."""
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
