"""Multi-GPU behind the C ABI (bm_options.devices): one process, several band
devices, the frame gathered into the root's render target.

On this one-GPU box every band device is device 0 (bm_options allows repeats: each band source still
gets its own context, stream, replicated meshes/scene/camera and band buffer, and the peer-write
gather kernel runs exactly as on 8 GPUs, minus the xGMI hop). Bar: every plane of the gathered frame
bit-identical to the single-device frame, which the config tests pin to the oracle.
"""
import os
import subprocess

import numpy as np
import pytest

from gpu_util import gpu_build, gpu_frame, oracle_frame
from raytracercuda_amd import beam, scenes

pytestmark = pytest.mark.gpu

LIGHT = (0.0, 10.0, -10.0)


def single_frame(meshes, w, h, cam, eye, orient, light=None):
    c = beam.Context(device=0)
    scene, keep, _ = gpu_build(c, meshes)
    cm = beam.ICamera.create(c)
    assert cm.setInitialRays(w, h, *cam) == 0
    rt = beam.IRenderTarget.createOffscreen(c, w, h)
    assert (cm.traceShadow(eye, orient, scene, rt, light) if light else cm.trace(eye, orient, scene, rt)) == 0
    f = rt.read(rgb=True)
    if light:
        f["shadow"] = rt.readShadow()
    rt.destroy()
    cm.destroy()
    scene.destroy()
    c.close()
    return f


@pytest.mark.parametrize("n,band,planes", [(3, 16, None), (5, 8, None), (8, 16, None),
                                           (4, 16, ["packed", "tri_id", "t", "nz", "shadow"])])
def test_bunny_1080_shadow_frame_over_n_devices(n, band, planes):
    """Default exchange: triangle ids (+ shadow bytes) travel and the root rebuilds t, |n.z| and the
    packed colour from them; with an explicit plane mask every plane travels as traced."""
    meshes = scenes.load_mesh("bunny")
    ref = single_frame(meshes, 1920, 1080, scenes.RAYS_1080, scenes.BUNNY_EYE, scenes.IDENTITY, LIGHT)
    ctx = beam.Context(device=0, devices=[0] * n, band_height=band, planes=planes)
    scene, keep, _ = gpu_build(ctx, meshes)
    cam = beam.ICamera.create(ctx)
    assert cam.setInitialRays(1920, 1080, *scenes.RAYS_1080) == 0
    rt = beam.IRenderTarget.createOffscreen(ctx, 1920, 1080)
    for _ in range(2):  # the second frame reuses the band buffers
        assert cam.traceShadow(scenes.BUNNY_EYE, scenes.IDENTITY, scene, rt, LIGHT) == 0
        f = rt.read(rgb=True)
        for k in ("packed", "tri_id", "t", "rgb"):
            assert np.array_equal(f[k], ref[k]), k
        assert np.array_equal(rt.readShadow(), ref["shadow"])
        assert cam.trace(scenes.BUNNY_EYE, scenes.IDENTITY, scene, rt) == 0  # primary only
        assert np.array_equal(rt.read()["tri_id"], ref["tri_id"])
    rt.destroy()
    cam.destroy()
    scene.destroy()
    ctx.close()


def test_gather_planes_mask_and_ragged_frame(oracle):
    """Only the planes in the mask are gathered (the others keep what they held); a frame whose
    height is no multiple of the band height and smaller than one band per device."""
    meshes = scenes.load_mesh("suzanne")
    w, h, eye = 77, 45, (0.0, 0.0, -3.0)
    packed, tri, t = oracle_frame(oracle, meshes, w, h, scenes.RAYS_SQUARE, eye, scenes.IDENTITY)
    ctx = beam.Context(device=0, devices=[0] * 4, planes=["packed"])
    scene, keep, _ = gpu_build(ctx, meshes)
    cam = beam.ICamera.create(ctx)
    assert cam.setInitialRays(w, h, *scenes.RAYS_SQUARE) == 0
    rt = beam.IRenderTarget.createOffscreen(ctx, w, h)
    assert rt.lock() == 0
    assert cam.clear(0x00123456) == 0
    assert cam.traceScene(eye, scenes.IDENTITY, scene) == 0
    f = {k: v.reshape(-1) for k, v in rt.read().items()}
    assert np.array_equal(f["packed"], packed)
    assert rt.unlock() == 0
    rt.destroy()
    cam.destroy()
    scene.destroy()
    ctx.close()
    full = beam.Context(device=0, devices=[0] * 4, band_height=4)
    scene, keep, _ = gpu_build(full, meshes)
    f = gpu_frame(full, scene, w, h, scenes.RAYS_SQUARE, eye, scenes.IDENTITY)
    assert np.array_equal(f["packed"], packed) and np.array_equal(f["tri_id"], tri) and np.array_equal(f["t"], t)
    scene.destroy()
    full.close()


def test_frames_in_flight_rebuild_and_refit():
    """Two render targets on their own streams, a rebuild with a larger scene right after traces on
    those streams (buffers grow under in-flight work), then a refit: every frame equals the
    single-device frame of the same geometry."""
    import torch
    small, big = scenes.load_mesh("suzanne"), scenes.scene("armadillo_proxy")
    eye = scenes.BUNNY_EYE
    ctx = beam.Context(device=0, devices=[0, 0, 0])
    scene = beam.IScene.create(ctx)
    keep = beam.upload_meshes(ctx, scene, small)
    scene.updateGPUScene()
    cam = beam.ICamera.create(ctx)
    assert cam.setInitialRays(640, 360, *scenes.RAYS_1080) == 0
    streams = [torch.cuda.Stream(device=0) for _ in range(2)]
    rts = [beam.IRenderTarget.createOffscreen(ctx, 640, 360) for _ in range(2)]
    for rt, st in zip(rts, streams):
        rt.setStream(st.cuda_stream)
    for _ in range(3):
        for rt in rts:
            assert cam.trace(eye, scenes.IDENTITY, scene, rt) == 0
    ref_small = single_frame(small, 640, 360, scenes.RAYS_1080, eye, scenes.IDENTITY)
    for rt in rts:
        assert np.array_equal(rt.read()["tri_id"], ref_small["tri_id"])
    # rebuild with 18x the triangles while the targets' streams may still be busy
    for rt in rts:
        assert cam.trace(eye, scenes.IDENTITY, scene, rt) == 0
    scene.removeMesh(keep[0])
    keep2 = beam.upload_meshes(ctx, scene, big)
    scene.updateGPUScene()
    ref_big = single_frame(big, 640, 360, scenes.RAYS_1080, eye, scenes.IDENTITY)
    for rt in rts:
        assert cam.trace(eye, scenes.IDENTITY, scene, rt) == 0
        f = rt.read()
        assert np.array_equal(f["tri_id"], ref_big["tri_id"]) and np.array_equal(f["t"], ref_big["t"])
    # refit with moved vertices on every replica
    moved = [dict(m, pos=(m["pos"] + np.float32([0.01, 0.0, 0.0])).astype(np.float32)) for m in big]
    for gm, m in zip(keep2, moved):
        assert gm.setVertexData(m["pos"], m["pos"].shape[0], 3, beam.VERTEX_DATA_POSITION) == 0
    scene.refitGPUScene()
    ref_moved = single_frame(moved, 640, 360, scenes.RAYS_1080, eye, scenes.IDENTITY)
    for rt in rts:
        assert cam.trace(eye, scenes.IDENTITY, scene, rt) == 0
        assert np.array_equal(rt.read()["tri_id"], ref_moved["tri_id"])
    for rt in rts:
        rt.destroy()
    cam.destroy()
    scene.destroy()
    ctx.close()


def test_lazy_original_records_ordered_across_render_target_streams():
    """a scene built without the original-order triangle records — the path of a scene
    built before bm_context_start_comm, forced here by the BM_PARAM_ORIG_LAZY test hook — gets them from
    the first multi-device trace, on that render target's stream. A second target on another stream must
    not reshade from them before that launch has written them. Every plane the root rebuilds from the ids
    (t, packed, rgb) equals the single-device frame on both targets, after the build and after a rebuild
    (which invalidates the records again)."""
    import torch
    meshes = scenes.scene("armadillo_proxy")
    ref = single_frame(meshes, 1920, 1080, scenes.RAYS_1080, scenes.BUNNY_EYE, scenes.IDENTITY)
    ctx = beam.Context(device=0, devices=[0, 0], params={"orig_lazy": 1})
    scene, keep, _ = gpu_build(ctx, meshes)
    cam = beam.ICamera.create(ctx)
    assert cam.setInitialRays(1920, 1080, *scenes.RAYS_1080) == 0
    streams = [torch.cuda.Stream(device=0) for _ in range(2)]
    rts = [beam.IRenderTarget.createOffscreen(ctx, 1920, 1080) for _ in range(2)]
    for rt, st in zip(rts, streams):
        rt.setStream(st.cuda_stream)
    for rep in range(2):
        if rep:
            scene.updateGPUScene()
        for rt in rts:  # back to back: the second target's trace is enqueued while the first still runs
            assert cam.trace(scenes.BUNNY_EYE, scenes.IDENTITY, scene, rt) == 0
        for rt in rts:
            f = rt.read(rgb=True)
            for k in ("packed", "tri_id", "t", "rgb"):
                assert np.array_equal(f[k], ref[k]), (rep, k)
    for rt in rts:
        rt.destroy()
    cam.destroy()
    scene.destroy()
    del keep
    ctx.close()


@pytest.mark.parametrize("n,band,planes,light,size", [
    (2, 16, None, None, (1920, 1080)),                       # by id: the root reshades
    (4, 16, ["packed", "tri_id", "t", "nz"], None, (1920, 1080)),
    (3, 16, None, LIGHT, (1920, 1080)),                      # ids + u8 shadow bytes
    (8, 16, ["packed", "tri_id", "t", "nz", "shadow"], LIGHT, (1920, 1080)),
    (3, 5, None, None, (77, 45)),                            # ragged: rows * W odd, < one band per source
    (5, 3, ["packed", "tri_id", "t", "nz", "shadow"], LIGHT, (77, 45)),
    (2, 5, ["packed", "tri_id", "t", "nz"], LIGHT, (77, 45)),  # shadow bytes left out of the mask
])
def test_rccl_gather_on_one_gpu(n, band, planes, light, size):
    """The RCCL transport executed on the one-GPU box: a repeated device list with gather="rccl" runs
    one single-rank communicator (bm_comm_unique_id's path: ncclGetUniqueId + ncclCommInitRank) and
    every band source's planes travel by grouped ncclSend/ncclRecv to itself into the root's staging
    area, then the multi-source k_band_scatter (blockIdx.z > 0) places them — the code of the
    multi-GPU RCCL gather minus the xGMI hop. Every plane equals the single-device frame."""
    w, h = size
    meshes = scenes.load_mesh("bunny")
    ref = single_frame(meshes, w, h, scenes.RAYS_1080, scenes.BUNNY_EYE, scenes.IDENTITY, light)
    ctx = beam.Context(device=0, devices=[0] * n, band_height=band, planes=planes, gather="rccl")
    assert ctx.gather == "rccl-loopback"
    scene, keep, _ = gpu_build(ctx, meshes)
    cam = beam.ICamera.create(ctx)
    assert cam.setInitialRays(w, h, *scenes.RAYS_1080) == 0
    rt = beam.IRenderTarget.createOffscreen(ctx, w, h)
    for _ in range(2):  # the second frame reuses staging and band buffers
        err = (cam.traceShadow(scenes.BUNNY_EYE, scenes.IDENTITY, scene, rt, light) if light else
               cam.trace(scenes.BUNNY_EYE, scenes.IDENTITY, scene, rt))
        assert err == 0, ctx.last_error()
        f = rt.read(rgb=True)
        for k in ("packed", "tri_id", "t", "rgb"):
            assert np.array_equal(f[k], ref[k]), k
        if light and (planes is None or "shadow" in planes):
            assert np.array_equal(rt.readShadow(), ref["shadow"])
    rt.destroy()
    cam.destroy()
    scene.destroy()
    ctx.close()


def test_multi_device_errors():
    with pytest.raises(beam.BeamError):  # reference modes trace whole frames on one device
        beam.Context(device=0, devices=[0, 0], reference_kd=True, gather="rccl")
    with pytest.raises(beam.BeamError):  # reference modes trace whole frames on one device
        beam.Context(device=0, devices=[0, 0], reference_kd=True)
    with pytest.raises(beam.BeamError):
        beam.Context(device=0, devices=[0] * 9)
    ctx = beam.Context(device=0, devices=[0, 0])
    other = beam.Context(device=0)
    scene = beam.IScene.create(ctx)
    scene.updateGPUScene()
    cam = beam.ICamera.create(ctx)
    assert cam.setInitialRays(32, 32) == 0
    rt_other = beam.IRenderTarget.createOffscreen(other, 32, 32)
    assert cam.trace((0, 0, -3), scenes.IDENTITY, scene, rt_other) == beam.ERROR_INVALID_PARAMETER
    rt = beam.IRenderTarget.createOffscreen(ctx, 32, 16)
    assert cam.trace((0, 0, -3), scenes.IDENTITY, scene, rt) == beam.ERROR_RT_CAM_MISMATCH
    rt2 = beam.IRenderTarget.createOffscreen(ctx, 32, 32)
    unbuilt = beam.IScene.create(ctx)
    assert cam.trace((0, 0, -3), scenes.IDENTITY, unbuilt, rt2) == beam.ERROR_NOT_BUILT
    assert cam.trace((0, 0, -3), scenes.IDENTITY, scene, rt2) == 0  # empty scene: every pixel misses
    assert (rt2.read()["tri_id"] == 0xFFFFFFFF).all()
    for h in (rt, rt2, rt_other, cam, scene, unbuilt):
        h.destroy()
    ctx.close()
    other.close()


def test_cpp_example_on_a_device_list(tmp_path):
    """examples/render_offscreen with a device list (Beam::setDevices): the TestProgram-shaped C++
    caller renders over 4 band devices without Python, and its frame equals the 1-device run."""
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "examples", "render_offscreen")
    if not os.path.exists(exe):
        subprocess.run(["make", "-s", "-C", os.path.dirname(exe)], check=True)
    outs = []
    for devs in (None, "0,0,0,0"):
        out = tmp_path / f"f{len(outs)}.ppm"
        r = subprocess.run([exe, str(out)] + ([devs] if devs else []), capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr
        assert ("on 4 device(s)" if devs else "on 1 device(s)") in r.stdout
        outs.append(out.read_bytes())
    assert outs[0] == outs[1]
