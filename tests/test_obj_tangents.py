"""Tangent space of the OBJ ingest (host-only): the slots Model::load fills from Assimp's
aiProcess_CalcTangentSpace (TestProgram/Model.cpp:34 asks for it, :107-113 uploads mTangents /
mBitangents into VERTEX_DATA_TANGENT / BITANGENT).

Assimp is absent from the reference (a Windows DLL, no source), so this boundary is "parity unpinned":
`reference_tangents` below restates Assimp's published CalcTangentsProcess independently of
csrc/bm_obj.cpp — numpy float32, one IEEE operation per step, in the order bm_obj.cpp documents — and
the native reader must give the same tangent and bitangent bits on every corner.
"""
import numpy as np
import pytest

from raytracercuda_amd import beam, scenes

F = np.float32


def _norm_safe(a):
    ln = np.sqrt(F(a[0] * a[0] + a[1] * a[1]) + F(a[2] * a[2]))  # (x*x + y*y) + z*z, then sqrt
    if not ln > F(0):
        return a
    inv = F(F(1) / ln)
    return np.array([a[0] * inv, a[1] * inv, a[2] * inv], F)


def _norm(a):
    ln = np.sqrt(F(a[0] * a[0] + a[1] * a[1]) + F(a[2] * a[2]))
    if ln == F(0):
        return a
    inv = F(F(1) / ln)
    return np.array([a[0] * inv, a[1] * inv, a[2] * inv], F)


def _dot(a, b):
    return F(F(a[0] * b[0] + a[1] * b[1]) + F(a[2] * b[2]))


def _cross(a, b):
    return np.array([a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]], F)


def reference_tangents(P, N, U):
    """Assimp's CalcTangentsProcess over unshared corners (3 per triangle): per-face tangent and
    bitangent from the UV gradients, projected into each corner's normal plane, then smoothed over
    corners at the same position (SpatialSort radius 1e-4 x the bounding-box diagonal) whose normals
    agree to 0.9999 and tangents and bitangents to cos 45 deg."""
    P, N, U = (np.asarray(x, F) for x in (P, N, U))
    nc = P.shape[0]
    T = np.zeros((nc, 3), F)
    B = np.zeros((nc, 3), F)
    with np.errstate(all="ignore"):
        for f in range(0, nc - 2, 3):
            v, w = P[f + 1] - P[f], P[f + 2] - P[f]
            sx, sy = U[f + 1, 0] - U[f, 0], U[f + 1, 1] - U[f, 1]
            tx, ty = U[f + 2, 0] - U[f, 0], U[f + 2, 1] - U[f, 1]
            d = F(-1) if F(tx * sy) - F(ty * sx) < 0 else F(1)
            if F(sx * ty) == F(sy * tx):
                sx, sy, tx, ty = F(0), F(1), F(1), F(0)
            tg = np.array([F(w[c] * sy) - F(v[c] * ty) for c in range(3)], F) * d
            bt = np.array([F(w[c] * sx) - F(v[c] * tx) for c in range(3)], F) * d
            for p in range(f, f + 3):
                lt = _norm_safe(tg - N[p] * _dot(tg, N[p]))
                lb = _norm_safe(bt - N[p] * _dot(bt, N[p]))
                it, ib = not np.all(np.isfinite(lt)), not np.all(np.isfinite(lb))
                if it != ib:
                    if it:
                        lt = _norm_safe(_cross(N[p], lb))
                    else:
                        lb = _norm_safe(_cross(lt, N[p]))
                T[p], B[p] = lt, lb
        ext = P.max(0) - P.min(0)
        eps = F(np.sqrt(_dot(ext, ext)) * F(1e-4))
        eps2 = F(eps * eps)
        pn = _norm(np.array([0.8523, 0.0812, 0.5165], F))
        dist = np.array([_dot(P[i], pn) for i in range(nc)], F)
        order = np.argsort(dist, kind="stable")
        sd = dist[order]
        limit = F(np.cos(F(F(45) * F(0.0174532925))))
        done = np.zeros(nc, bool)
        for a in range(nc):
            if done[a]:
                continue
            pa, na, ta, ba = P[a].copy(), N[a].copy(), T[a].copy(), B[a].copy()
            group = [a]
            k = int(np.searchsorted(sd, F(dist[a] - eps), side="left"))
            while k < nc and sd[k] < F(dist[a] + eps):
                j = int(order[k])
                k += 1
                dp = P[j] - pa
                if not _dot(dp, dp) < eps2 or done[j]:
                    continue
                if _dot(N[j], na) < F(0.9999) or _dot(T[j], ta) < limit or _dot(B[j], ba) < limit:
                    continue
                group.append(j)
                done[j] = True
            st = np.zeros(3, F)
            sb = np.zeros(3, F)
            for j in group:
                st = st + T[j]
                sb = sb + B[j]
            st, sb = _norm(st), _norm(sb)
            for j in group:
                T[j], B[j] = st, sb
    return T, B


def write_obj(path, pos, nrm, uv, tris):
    lines = ["o part"]
    lines += ["v " + " ".join(repr(float(x)) for x in p) for p in pos]
    lines += ["vn " + " ".join(repr(float(x)) for x in n) for n in nrm]
    lines += ["vt " + " ".join(repr(float(x)) for x in t) for t in uv]
    lines.append("usemtl m")
    lines += ["f " + " ".join(f"{i + 1}/{i + 1}/{i + 1}" for i in t) for t in tris]
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")


def corner_arrays(pos, nrm, uv, tris):
    c = np.asarray(tris, np.int64).reshape(-1)
    return np.asarray(pos, F)[c], np.asarray(nrm, F)[c], np.asarray(uv, F)[c]


def check(path, pos, nrm, uv, tris):
    want_t, want_b = reference_tangents(*corner_arrays(pos, nrm, uv, tris))
    for unshared in (False, True):
        m = beam.Model(path, unshared=unshared)
        (g,) = m.meshes()
        m.destroy()
        assert g["tan"] is not None and g["bit"] is not None
        assert g["tan"].shape == g["pos"].shape == g["bit"].shape
        got_t, got_b = g["tan"][g["idx"].astype(np.int64)], g["bit"][g["idx"].astype(np.int64)]
        assert np.array_equal(got_t.view(np.uint32), want_t.view(np.uint32)), \
            f"{int((got_t != want_t).any(1).sum())} corner tangents differ"
        assert np.array_equal(got_b.view(np.uint32), want_b.view(np.uint32))
        # positions, normals and UVs per corner are still the file's
        p, n, u = corner_arrays(pos, nrm, uv, tris)
        assert np.array_equal(g["pos"][g["idx"].astype(np.int64)], p)
        assert np.array_equal(g["nrm"][g["idx"].astype(np.int64)], n)
        assert np.array_equal(g["uv"][g["idx"].astype(np.int64)], u)
        if unshared:
            assert g["pos"].shape[0] == len(tris) * 3
    return g


def test_tangents_f16_fixture(tmp_path):
    """The f16 fixture's first mesh (1,852 triangles) with a synthetic UV layout."""
    f16 = scenes.load_mesh("f16")[0]
    pos, nrm, tris = f16["pos"], f16["nrm"], np.asarray(f16["idx"]).reshape(-1, 3)
    i = np.arange(pos.shape[0])
    uv = np.stack([np.sin(i * 0.37), np.cos(i * 0.11) * 0.5], 1).astype(F)
    p = str(tmp_path / "f16.obj")
    write_obj(p, pos, nrm, uv, tris)
    check(p, pos, nrm, uv, tris)


def test_tangents_degenerate_uv_and_mirrored_seams(tmp_path):
    """A grid whose left half has its U mirrored (tangents flip across the seam: the seam corners must
    not share a vertex or a tangent) plus a strip with all-equal UVs (no UV gradient: Assimp's
    default direction) and unnormalised normals."""
    n = 6
    pos, nrm, uv, tris = [], [], [], []
    for y in range(n + 1):
        for x in range(n + 1):
            pos.append([x * 0.5, y * 0.5, 0.1 * np.sin(x + y)])
            nrm.append([0.05 * x, 0.0, 2.0])  # not unit length
            u = x / n if x >= n // 2 else (n - x) / n  # mirrored at the centre column
            uv.append([u, y / n])
    for y in range(n):
        for x in range(n):
            a = y * (n + 1) + x
            tris += [[a, a + 1, a + n + 2], [a, a + n + 2, a + n + 1]]
    base = len(pos)
    for k in range(4):  # a strip with one UV for every corner
        pos.append([k * 0.3, -1.0, 0.0])
        pos.append([k * 0.3, -1.5, 0.2])
        nrm += [[0.0, 0.3, 1.0], [0.0, 0.3, 1.0]]
        uv += [[0.25, 0.25], [0.25, 0.25]]
    for k in range(3):
        a = base + 2 * k
        tris += [[a, a + 2, a + 1], [a + 1, a + 2, a + 3]]
    pos, nrm, uv = np.float32(pos), np.float32(nrm), np.float32(uv)
    p = str(tmp_path / "grid.obj")
    write_obj(p, pos, nrm, uv, tris)
    g = check(p, pos, nrm, uv, tris)
    # the shared layout: a (v, vt, vn) triple whose corners got different tangents is split
    triples = len(set(np.asarray(tris).reshape(-1).tolist()))
    assert g["pos"].shape[0] > triples


def test_no_tangents_without_uv_or_normals(tmp_path):
    p = tmp_path / "nouv.obj"
    p.write_text("v 0 0 0\nv 1 0 0\nv 0 1 0\nvn 0 0 1\nf 1//1 2//1 3//1\n")
    m = beam.Model(str(p))
    (g,) = m.meshes()
    m.destroy()
    assert g["uv"] is None and g["tan"] is None and g["bit"] is None
    q = tmp_path / "nonrm.obj"
    q.write_text("v 0 0 0\nv 1 0 0\nv 0 1 0\nvt 0 0\nvt 1 0\nvt 0 1\nf 1/1 2/2 3/3\n")
    m = beam.Model(str(q))
    (g,) = m.meshes()
    m.destroy()
    assert g["nrm"] is None and g["tan"] is None
