"""OBJ ingest: the native reader behind Model::load (csrc/bm_obj.cpp) — host-only,
so these run without a GPU.

Parity status at this boundary is "unpinned" against Assimp (absent from the reference); the pins are
oracle/beam_oracle.c's reader (which produced the golden meshes) and, in tests/test_gpu_parity.py,
the golden frames. What the hot path sees is compared: per-triangle corner positions and normals
(de-indexed) bit for bit, mesh split, face order.
"""
import os
import tempfile
import zipfile

import numpy as np
import pytest

from raytracercuda_amd import beam, scenes

REF_CONTENT = "/root/reference/Content"


def corners(meshes, key="pos"):
    """Per-triangle corner attributes, concatenated over meshes (the order the build numbers ids)."""
    out = []
    for m in meshes:
        a = m[key]
        out.append(np.asarray(a, np.float32)[np.asarray(m["idx"], np.int64)].reshape(-1, 3, a.shape[1]))
    return np.concatenate(out) if out else np.zeros((0, 3, 3), np.float32)


def write_obj(path, meshes, quads=False, negative=False):
    """An OBJ with v/vt/vn triplets, one usemtl run per mesh, comments and ignored statements."""
    lines = ["# synthetic fixture", "mtllib none.mtl", "s off"]
    nv = 0
    for k, m in enumerate(meshes):
        pos, nrm = np.asarray(m["pos"], np.float32), np.asarray(m["nrm"], np.float32)
        idx = np.asarray(m["idx"], np.int64).reshape(-1, 3)
        lines.append(f"o part{k}")
        for p in pos:
            lines.append("v " + " ".join(repr(float(x)) for x in p))
        for n in nrm:
            lines.append("vn " + " ".join(repr(float(x)) for x in n))
        for i in range(pos.shape[0]):
            lines.append(f"vt {i % 7 / 7.0} {i % 5 / 5.0}")
        lines.append(f"usemtl mat{k}")
        base = nv
        for t in idx:
            if negative:
                ref = [str(int(i) - pos.shape[0]) for i in t]  # relative to this mesh's block
                lines.append("f " + " ".join(f"{r}/{r}/{r}" for r in ref))
            else:
                ref = [str(base + int(i) + 1) for i in t]
                lines.append("f " + " ".join(f"{r}/{r}/{r}" for r in ref))
        nv += pos.shape[0]
    if quads:
        # one extra quad in its own material run: becomes the fan (0,1,2), (0,2,3)
        lines += ["usemtl quad", "v 0 0 0", "v 1 0 0", "v 1 1 0", "v 0 1 0", "vn 0 0 1",
                  "f -4//1 -3//1 -2//1 -1//1"]
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")


@pytest.fixture(scope="module")
def f16():
    return scenes.load_mesh("f16")


@pytest.mark.parametrize("negative", [False, True])
def test_synthetic_obj_round_trip(tmp_path, f16, negative):
    p = str(tmp_path / "f16.obj")
    write_obj(p, f16, quads=True, negative=negative)
    for unshared in (False, True):
        m = beam.Model(p, unshared=unshared)
        got = m.meshes()
        info = m.info()
        m.destroy()
        assert [g["material"] for g in got] == ["mat0", "mat1", "quad"]
        assert info["num_meshes"] == 3 and info["num_faces"] == sum(x["idx"].size // 3 for x in f16) + 2
        for a, b in zip(got[:2], f16):
            assert np.array_equal(corners([a]), corners([b]))
            assert np.array_equal(corners([a], "nrm"), corners([b], "nrm"))
            assert a["uv"] is not None and a["uv"].shape == (a["pos"].shape[0], 2)
        q = got[2]
        assert np.array_equal(corners([q]), np.float32([[[0, 0, 0], [1, 0, 0], [1, 1, 0]],
                                                        [[0, 0, 0], [1, 1, 0], [0, 1, 0]]]))
        assert q["uv"] is None  # the quad's corners have no vt
        if unshared:
            assert all(g["pos"].shape[0] == g["idx"].size for g in got)
        else:  # equal index triples share a vertex: the quad's fan reuses corners 0 and 2
            assert q["pos"].shape[0] == 4 and q["idx"].size == 6


def test_reader_errors(tmp_path):
    with pytest.raises(beam.BeamError):
        beam.Model(str(tmp_path / "missing.obj"))
    bad = tmp_path / "bad.obj"
    bad.write_text("v 0 0 0\nv 1 0 0\nv 0 1 0\nf 1 2 x\n")
    with pytest.raises(beam.BeamError) as e:
        beam.Model(str(bad))
    assert e.value.code == beam.ERROR_INVALID_FORMAT
    empty = tmp_path / "empty.obj"
    empty.write_text("# nothing\nv 0 0 0\n")
    m = beam.Model(str(empty))
    assert m.info()["num_meshes"] == 0
    m.destroy()


@pytest.mark.skipif(not os.path.isdir(REF_CONTENT), reason="reference content not present on this host")
@pytest.mark.parametrize("name", ["suzanne", "f16", "bunny"])
def test_reference_content_matches_oracle_reader(oracle, name):
    """The reference's own Content files: native reader == the oracle reader that made the fixtures."""
    with tempfile.TemporaryDirectory() as tmp:
        if name == "bunny":
            with zipfile.ZipFile(os.path.join(REF_CONTENT, "bunny.zip")) as z:
                z.extract("bunny.obj", tmp)
            path = os.path.join(tmp, "bunny.obj")
        else:
            path = os.path.join(REF_CONTENT, name + ".obj")
        m = beam.Model(path)
        got = m.meshes()
        m.destroy()
        ref = oracle.load_obj(path, share=0)  # unshared corners, normals vn[ni]
    assert len(got) == len(ref)
    assert np.array_equal(corners(got), corners(ref))
    assert np.array_equal(corners(got, "nrm"), corners(ref, "nrm"))
    if name != "suzanne":  # the committed suzanne fixture follows the survey's vn[vi] convention
        assert np.array_equal(corners(got), corners(scenes.load_mesh(name)))
        assert np.array_equal(corners(got, "nrm"), corners(scenes.load_mesh(name), "nrm"))


@pytest.mark.gpu
@pytest.mark.parametrize("num_adds", [1, 2])
def test_model_load_renders_golden_frame(tmp_path, f16, num_adds):
    """Model::load through the native reader into a scene; the f16 golden view renders bit-exact.
    numAdds=2 adds every mesh twice in a row (Model.cpp:52-54: mesh0, mesh0, mesh1, mesh1): the
    copies tie exactly and the lower (first) copy's triangle ids win."""
    from golden_io import closest_hit_expected, manifest, view
    p = str(tmp_path / "f16.obj")
    write_obj(p, f16)
    ctx = beam.Context(device=0)
    scene = beam.IScene.create(ctx)
    model = beam.Model.load(ctx, p, scene, num_adds)
    st = scene.updateGPUScene(stats=True)
    assert st["num_meshes"] == 2 * num_adds and st["num_tris"] == 4056 * num_adds
    m = manifest()["views"]["f16_500"]
    cam = beam.ICamera.create(ctx)
    assert cam.setInitialRays(m["w"], m["h"], *m["rays"]) == 0
    rt = beam.IRenderTarget.createOffscreen(ctx, m["w"], m["h"])
    assert cam.trace(m["eye"], scenes.IDENTITY, scene, rt) == 0
    f = rt.read()
    packed, tri, t = closest_hit_expected(m["w"] * m["h"], view("f16_500"))
    n0 = f16[0]["idx"].size // 3  # mesh 1's ids move past mesh 0's extra copies
    tri = np.where((tri != 0xFFFFFFFF) & (tri >= n0), tri + (num_adds - 1) * n0, tri).astype(np.uint32)
    assert np.array_equal(f["tri_id"].reshape(-1), tri)
    assert np.array_equal(f["packed"].reshape(-1), packed)
    rt.destroy()
    cam.destroy()
    scene.destroy()
    model.destroy()
    ctx.close()
