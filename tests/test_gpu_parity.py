"""GPU parity: the HIP path (through the C ABI) against the oracle and the golden frames.

Bars (BASELINE.json north_star): triangle ids and packed colours bit-exact; t and rgb within 1e-5
(t is in fact bit-exact: same operations, no contraction). The BASELINE configs (C1-C5, reference-mode golden frames) live in
test_gpu_00_configs.py, collected first.
"""
import numpy as np
import pytest

from golden_io import closest_hit_expected, manifest, sweep
from gpu_util import assert_frame_equal, gpu_build, gpu_frame, oracle_frame
from raytracercuda_amd import beam, scenes

pytestmark = pytest.mark.gpu

@pytest.mark.parametrize("name,leaf,width", [("bunny", 4, 4), ("bunny", 4, 2), ("suzanne", 1, 4), ("suzanne", 1, 2),
                                             ("f16", 16, 4), ("armadillo_proxy", 4, 4), ("armadillo_proxy", 4, 2),
                                             ("merged_proxy", 4, 4), ("merged_proxy", 4, 2)])
def test_bvh_build_bit_identical_to_oracle(oracle, name, leaf, width):
    meshes = scenes.scene(name)
    c2 = beam.Context(device=0, leaf_size=leaf, bvh_width=width)
    scene, keep, stats = gpu_build(c2, meshes)
    assert stats["bvh_width"] == width
    rec, tris, keys, perm = scene.export()
    orec, otris, okeys, operm = oracle.bvh_build(meshes, leaf, width).export()
    assert stats["num_tris"] == okeys.size
    assert np.array_equal(keys, okeys)
    assert np.array_equal(perm, operm)
    assert np.array_equal(tris, otris)
    assert rec.shape == orec.shape
    if width == 2:
        assert np.array_equal(rec, orec), f"{int((rec != orec).any(1).sum())} records differ"
    else:  # BVH4 writes only the slots a traversal reaches
        reach = beam.reachable_records(orec)
        assert np.array_equal(reach, beam.reachable_records(rec))
        assert np.array_equal(rec[reach], orec[reach]), f"{int((rec[reach] != orec[reach]).any(1).sum())} differ"
    scene.destroy()
    c2.close()


def test_camera_sweep(ctx):
    s = sweep()
    scene, keep, _ = gpu_build(ctx, scenes.load_mesh("bunny"))
    for k in range(s["eyes"].shape[0]):
        rec = {key[: -len(f"_{k}")]: v for key, v in s.items() if key.endswith(f"_{k}")}
        f = gpu_frame(ctx, scene, 128, 128, scenes.RAYS_SQUARE, s["eyes"][k], s["orients"][k])
        assert_frame_equal(f, *closest_hit_expected(128 * 128, rec))
    scene.destroy()


def test_multi_mesh_ids_and_proxy_scene(ctx, oracle):
    meshes = scenes.load_mesh("f16") + scenes.load_mesh("suzanne")
    scene, keep, st = gpu_build(ctx, meshes)
    assert st["num_meshes"] == 3 and st["num_tris"] == 3704 + 352 + 15488
    eye = (0.0, 0.0, -3.0)
    f = gpu_frame(ctx, scene, 200, 150, scenes.RAYS_1080, eye, scenes.IDENTITY)
    assert_frame_equal(f, *oracle_frame(oracle, meshes, 200, 150, scenes.RAYS_1080, eye, scenes.IDENTITY))
    scene.destroy()


def test_counters_match_oracle_traversal(ctx, oracle):
    m = manifest()["views"]["bunny_256"]
    meshes = scenes.load_mesh("bunny")
    scene, keep, _ = gpu_build(ctx, meshes)
    cam = beam.ICamera.create(ctx)
    assert cam.setInitialRays(m["w"], m["h"], *m["rays"]) == 0
    rt = beam.IRenderTarget.createOffscreen(ctx, m["w"], m["h"])
    cnt = cam.traceCounters(m["eye"], scenes.IDENTITY, scene, rt)
    err, rays = oracle.camera_rays(m["w"], m["h"], *m["rays"])
    _, _, _, ocnt = oracle.bvh_build(meshes, 4, ctx.bvh_width).render(rays, m["eye"], scenes.IDENTITY,
                                                                        counters=True)
    assert list(cnt) == list(ocnt)
    rt.destroy()
    cam.destroy()
    scene.destroy()


# ---- edge cases the reference's own behaviour defines -------------------------------------------
def test_empty_scene_all_miss(ctx):
    scene = beam.IScene.create(ctx)
    st = scene.updateGPUScene(stats=True)
    assert st["num_tris"] == 0
    f = gpu_frame(ctx, scene, 40, 30, scenes.RAYS_SQUARE, (0, 0, -3), scenes.IDENTITY)
    assert np.all(f["packed"] == 0xFF00) and np.all(f["tri_id"] == 0xFFFFFFFF) and np.all(np.isinf(f["t"]))
    scene.destroy()


@pytest.mark.parametrize("ntri", [1, 2, 3, 5, 17])
def test_tiny_scenes_and_ragged_frames(ctx, oracle, ntri):
    rng = np.random.default_rng(ntri)
    pos = rng.uniform(-1, 1, size=(3 * ntri, 3)).astype(np.float32)
    nrm = rng.normal(size=(3 * ntri, 3)).astype(np.float32)
    meshes = [{"pos": pos, "nrm": nrm, "idx": np.arange(3 * ntri, dtype=np.uint32)}]
    scene, keep, _ = gpu_build(ctx, meshes)
    for w, h in [(1, 1), (17, 9), (37, 23)]:
        f = gpu_frame(ctx, scene, w, h, scenes.RAYS_SQUARE, (0.1, 0.05, -3), scenes.IDENTITY)
        assert_frame_equal(f, *oracle_frame(oracle, meshes, w, h, scenes.RAYS_SQUARE, (0.1, 0.05, -3),
                                            scenes.IDENTITY))
    scene.destroy()


def test_degenerate_geometry_matches_oracle(ctx, oracle):
    pos = np.array([[0, 0, 1], [1, 0, 1], [0, 1, 1], [1, 1, 1], [2, 2, 1], [0.5, 0.5, 2],
                    [0, 0, 1], [1, 0, 1], [0, 1, 1]], np.float32)
    nrm = np.tile(np.array([[0, 0, -1]], np.float32), (pos.shape[0], 1))
    idx = np.array([0, 1, 2, 1, 3, 2, 0, 3, 4, 0, 0, 0, 6, 7, 8, 5, 5, 4], np.uint32)
    meshes = [{"pos": pos, "nrm": nrm, "idx": idx}]
    scene, keep, _ = gpu_build(ctx, meshes)
    f = gpu_frame(ctx, scene, 33, 17, scenes.RAYS_SQUARE, (0.5, 0.5, 0.0), scenes.IDENTITY)
    assert_frame_equal(f, *oracle_frame(oracle, meshes, 33, 17, scenes.RAYS_SQUARE, (0.5, 0.5, 0.0),
                                        scenes.IDENTITY))
    scene.destroy()


def test_pitch_is_honoured_and_clear(ctx):
    scene, keep, _ = gpu_build(ctx, scenes.load_mesh("suzanne"))
    cam = beam.ICamera.create(ctx)
    assert cam.setInitialRays(50, 40, *scenes.RAYS_SQUARE) == 0
    rt = beam.IRenderTarget.createOffscreen(ctx, 50, 40, pitch=50 * 4 + 64)
    assert rt.lock() == 0
    assert cam.clear(0x123456) == 0
    assert np.all(rt.read()["packed"] == 0x123456)
    assert cam.traceScene((0, 0, -3), scenes.IDENTITY, scene) == 0
    a = rt.read()
    b = gpu_frame(ctx, scene, 50, 40, scenes.RAYS_SQUARE, (0, 0, -3), scenes.IDENTITY)
    assert np.array_equal(a["packed"].reshape(-1), b["packed"])
    assert rt.unlock() == 0
    rt.destroy()
    cam.destroy()
    scene.destroy()


def read_ppm(path):
    """Minimal binary-P6 reader (header: magic, width, height, maxval; then raw R, G, B bytes)."""
    data = open(path, "rb").read()
    fields, pos = [], 0
    while len(fields) < 4:
        while data[pos:pos + 1].isspace():
            pos += 1
        end = pos
        while not data[end:end + 1].isspace():
            end += 1
        fields.append(data[pos:end])
        pos = end
    assert fields[0] == b"P6" and fields[3] == b"255"
    w, h = int(fields[1]), int(fields[2])
    return np.frombuffer(data[pos + 1:], np.uint8).reshape(h, w, 3)


def test_save_ppm_matches_packed_plane(ctx, tmp_path):
    """bm_rt_save_ppm: bytes R, G, B of 0x00RRGGBB, pitch removed, rows top down."""
    scene, keep, _ = gpu_build(ctx, scenes.load_mesh("suzanne"))
    cam = beam.ICamera.create(ctx)
    assert cam.setInitialRays(50, 40, *scenes.RAYS_SQUARE) == 0
    rt = beam.IRenderTarget.createOffscreen(ctx, 50, 40, pitch=50 * 4 + 64)
    assert cam.trace((0, 0, -3), scenes.IDENTITY, scene, rt) == 0
    packed = rt.read()["packed"]
    rt.savePPM(tmp_path / "frame.ppm")
    img = read_ppm(tmp_path / "frame.ppm")
    assert img.shape == (40, 50, 3)
    assert np.array_equal(img[..., 0], (packed >> 16) & 0xFF)
    assert np.array_equal(img[..., 1], (packed >> 8) & 0xFF)
    assert np.array_equal(img[..., 2], packed & 0xFF)
    assert (img[..., 0] > 0).any() and (img[..., 1] == 255).any()  # hits (red) and misses (green)
    with pytest.raises(beam.BeamError):
        rt.savePPM(tmp_path / "missing_dir" / "frame.ppm")
    rt.destroy()
    cam.destroy()
    scene.destroy()


def test_band_partition_reassembles_to_full_frame(ctx):
    from raytracercuda_amd import multigpu
    scene, keep, _ = gpu_build(ctx, scenes.load_mesh("bunny"))
    w, h, bh = 96, 70, 16
    full = gpu_frame(ctx, scene, w, h, scenes.RAYS_1080, scenes.BUNNY_EYE, scenes.IDENTITY)
    cam = beam.ICamera.create(ctx)
    assert cam.setInitialRays(w, h, *scenes.RAYS_1080) == 0
    for world in (2, 3, 8):
        rows = multigpu.rows_per_rank(h, bh, world)
        parts = []
        for r in range(world):
            rt = beam.IRenderTarget.createOffscreen(ctx, w, rows)
            assert cam.traceBands(scenes.BUNNY_EYE, scenes.IDENTITY, scene, rt, bh, world, r) == 0
            parts.append(np.stack([rt.read()["tri_id"]]))
            rt.destroy()
        frame = multigpu.reassemble_np(np.stack(parts), h, bh)[0]
        assert np.array_equal(frame.reshape(-1), full["tri_id"])
    cam.destroy()
    scene.destroy()


def test_error_codes_follow_the_reference(ctx):
    E = beam
    mesh = beam.IMesh.create(ctx)
    pos = np.zeros((3, 3), np.float32)
    assert mesh.setVertexData(pos, 3, 2, E.VERTEX_DATA_POSITION) == E.ERROR_INVALID_PARAMETER
    assert mesh.setIndices(np.arange(4, dtype=np.uint32), 4) == E.ERROR_INVALID_PARAMETER
    assert mesh.setIndices(np.array([0, 1, 5], np.uint32), 3) == 0
    assert mesh.setVertexData(pos, 3, 3, E.VERTEX_DATA_POSITION) == 0
    assert mesh.setVertexData(pos[:2], 2, 3, E.VERTEX_DATA_NORMAL) == E.ERROR_INVALID_PARAMETER
    scene = beam.IScene.create(ctx)
    scene.addMesh(mesh)
    with pytest.raises(beam.BeamError) as ei:  # no normals: the reference would crash (BuildTree.cu:489)
        scene.updateGPUScene()
    assert ei.value.code == 4
    assert mesh.setVertexData(pos, 3, 3, E.VERTEX_DATA_NORMAL) == 0
    with pytest.raises(beam.BeamError) as ei:  # index 5 >= 3 vertices
        scene.updateGPUScene()
    assert ei.value.code == E.ERROR_INVALID_PARAMETER
    cam = beam.ICamera.create(ctx)
    assert cam.setInitialRays(0, 4) == E.ERROR_INVALID_PARAMETER
    assert cam.setInitialRays(8, 8) == 0
    assert cam.traceScene((0, 0, 0), scenes.IDENTITY, scene) == E.ERROR_NO_RENDER_TARGET
    rt = beam.IRenderTarget.createOffscreen(ctx, 8, 9)
    assert rt.unlock() == E.ERROR_LOCK_FIRST
    assert rt.lock() == 0 and rt.lock() == E.ERROR_UNLOCK_FIRST
    assert cam.traceScene((0, 0, 0), scenes.IDENTITY, scene) == E.ERROR_RT_CAM_MISMATCH
    rt.unlock()
    rt.destroy()
    rt = beam.IRenderTarget.createOffscreen(ctx, 8, 8)
    assert cam.trace((0, 0, 0), scenes.IDENTITY, scene, rt) == 10  # not built
    rt.destroy()
    cam.destroy()
    scene.destroy()


def test_rebuild_after_remove_and_determinism(ctx):
    a, b = scenes.load_mesh("suzanne"), scenes.load_mesh("f16")
    scene = beam.IScene.create(ctx)
    ma = beam.upload_meshes(ctx, scene, a)
    mb = beam.upload_meshes(ctx, scene, b)
    scene.updateGPUScene(stats=True)
    r1 = scene.export()
    scene.updateGPUScene(stats=True)
    r2 = scene.export()
    for x, y in zip(r1, r2):
        assert np.array_equal(x, y)
    scene.removeMesh(ma[0])
    st = scene.updateGPUScene(stats=True)
    assert st["num_tris"] == 3704 + 352
    only_b = beam.IScene.create(ctx)
    keep = beam.upload_meshes(ctx, only_b, b)
    only_b.updateGPUScene(stats=True)
    (ra, *rest_a), (rb, *rest_b) = scene.export(), only_b.export()
    reach = beam.reachable_records(rb)  # a rebuilt BVH4 leaves stale data in unreachable slots
    assert np.array_equal(reach, beam.reachable_records(ra))
    assert np.array_equal(ra[reach], rb[reach])
    for x, y in zip(rest_a, rest_b):
        assert np.array_equal(x, y)
    scene.destroy()
    only_b.destroy()


def test_cpp_drop_in_example_matches_oracle(oracle, tmp_path):
    """examples/render_offscreen.cpp (reference-shaped C++ API, include/beam/Beam.h) end to end."""
    import os
    import subprocess
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "examples", "render_offscreen")
    if not os.path.exists(exe):
        subprocess.run(["make", "-s", "-C", os.path.dirname(exe)], check=True)
    out = tmp_path / "f.ppm"
    r = subprocess.run([exe, str(out)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    data = out.read_bytes()
    header_end = data.index(b"255\n") + 4
    rgb = np.frombuffer(data[header_end:], np.uint8).reshape(-1, 3).astype(np.uint32)
    packed = (rgb[:, 0] << 16) | (rgb[:, 1] << 8) | rgb[:, 2]
    pos = np.array([-1, -1, 1.56, 0, 1, 1.56, 1, -1, 1.56, 2, 1, 1.56], np.float32).reshape(4, 3)
    nrm = np.array([0, 0, -1, 0, 0, -1, 0, 0, -1, 0.3, 0, -1], np.float32).reshape(4, 3)
    meshes = [{"pos": pos, "nrm": nrm, "idx": np.array([0, 1, 2, 1, 2, 3], np.uint32)}]
    ep, et, ett = oracle_frame(oracle, meshes, 500, 500, scenes.RAYS_SQUARE, (0, 0, -2.1), scenes.IDENTITY)
    assert np.array_equal(packed, ep)
    assert int((et != 0xFFFFFFFF).sum()) > 0
