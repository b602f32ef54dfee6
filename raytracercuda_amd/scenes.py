"""Synthetic workloads of BASELINE.json's configs: committed meshes, deterministic proxies, views.

The reference ships bunny/f16/suzanne (Content/*.obj); armadillo.obj and tyra.obj are missing
(reference .MISSING_LARGE_BLOBS:3-8). SURVEY.md §8(d) defines deterministic proxies:

* armadillo proxy: bunny with one 1->4 midpoint subdivision (278,520 tris);
* tyra proxy: bunny subdivided twice (1,114,080 tris), merged with f16's two meshes for config 5.

Subdivision (float32, IEEE, operation order fixed here): midpoint = (a + b) * 0.5f; normal =
normalize(na + nb) with glm order (x*x + y*y) + z*z and v * (1/sqrt(.)); edge midpoints are
shared; per source face (a,b,c) the children are (a,ab,ca), (ab,b,bc), (ca,bc,c), (ab,bc,ca).
"""
from __future__ import annotations

import hashlib
import os

import numpy as np

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden")
MESH_DIR = os.path.join(GOLDEN_DIR, "meshes")

# Views (eye, camera rays) of SURVEY.md §8(c)/(d). Orient is the identity (column-major).
IDENTITY = np.eye(3, dtype=np.float32).reshape(9)
BUNNY_EYE = (-0.34, 1.2, -3.5)
RAYS_SQUARE = (-1.0, 1.0, -1.0, 1.0, 1.0)           # TestProgram convention (Program.cpp:189)
RAYS_1080 = (-1.7777778, 1.7777778, -1.0, 1.0, 1.0)  # 16:9
RAYS_4K = (-16.0 / 9.0, 16.0 / 9.0, -1.0, 1.0, 1.0)  # C4: rays(-16/9, 16/9, -1, 1, 1)
# Filled view (bench side figure): the eye close to the armadillo proxy, 85.5 % of the 1080p pixels
# hit (the reference camera's view of it hits 7.3 %), silhouettes included.
FILLED_EYE = (-0.3, 0.9, -0.9)
C5_LIGHT = (0.0, 10.0, -10.0)  # SURVEY §8(d) C5 point light

# BASELINE.json configs[1..4] (configs[0] is the CPU-only C1): scene, frame, camera rays, eye, light
CONFIGS = {
    "c2": {"scene": "bunny", "width": 1920, "height": 1080, "rays": RAYS_1080, "eye": BUNNY_EYE, "light": None},
    "c3": {"scene": "armadillo_proxy", "width": 1920, "height": 1080, "rays": RAYS_1080, "eye": BUNNY_EYE,
           "light": None},
    "c4": {"scene": "armadillo_proxy", "width": 3840, "height": 2160, "rays": RAYS_4K, "eye": BUNNY_EYE,
           "light": None},
    "c5": {"scene": "merged_proxy", "width": 1920, "height": 1080, "rays": RAYS_1080, "eye": BUNNY_EYE,
           "light": C5_LIGHT},
    "filled": {"scene": "armadillo_proxy", "width": 1920, "height": 1080, "rays": RAYS_1080, "eye": FILLED_EYE,
               "light": None},
    # the workload of the reference's only published timing (aa.xml: an Nsight profile of TestProgram on a
    # GTX 660 Ti — bmMarchKernel over 977 x 256 threads = 500x500 rays, the f16's two meshes inserted by two
    # bmInsertTriangleInTree launches of 15 and 2 blocks): Program.cpp:106,147,189's eye and camera rays
    "aa_xml": {"scene": "f16", "width": 500, "height": 500, "rays": RAYS_SQUARE, "eye": (0.0, 0.0, -2.1),
               "light": None},
}
# aa.xml's rows (bmInsertTriangleInTree 51,722.72 + 4,753.568 us; bmMarchKernel: mean of its 24 launches)
AA_XML_PUBLISHED = {"gpu": "GeForce GTX 660 Ti", "march_ms": 38.414, "build_ms": 51.72272 + 4.753568,
                    "source": "aa.xml rows bmInsertTriangleInTree x2, bmMarchKernel x24 (977 x 256 threads)"}


def load_mesh(name: str):
    """Load a committed mesh fixture (tests/golden/meshes/<name>.npz) as a list of meshes."""
    path = os.path.join(MESH_DIR, name + ".npz")
    with np.load(path, allow_pickle=False) as z:
        nm = int(z["num_meshes"])
        return [{"pos": z[f"pos{i}"], "nrm": z[f"nrm{i}"], "idx": z[f"idx{i}"]} for i in range(nm)]


def mesh_digest(meshes) -> str:
    h = hashlib.sha256()
    for m in meshes:
        for k in ("pos", "nrm", "idx"):
            a = m.get(k)
            if a is not None:
                h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def _normalize_rows(n: np.ndarray) -> np.ndarray:
    x, y, z = n[:, 0], n[:, 1], n[:, 2]
    d = (x * x + y * y) + z * z
    inv = np.float32(1.0) / np.sqrt(d)
    return (n * inv[:, None]).astype(np.float32)


def subdivide(mesh: dict) -> dict:
    """One 1->4 midpoint subdivision of a single indexed mesh (see module docstring)."""
    pos = np.asarray(mesh["pos"], np.float32)
    nrm = np.asarray(mesh["nrm"], np.float32)
    f = np.asarray(mesh["idx"], np.uint32).reshape(-1, 3).astype(np.int64)
    nv = pos.shape[0]
    a, b, c = f[:, 0], f[:, 1], f[:, 2]
    # edges in (ab, bc, ca) order per face, keyed by sorted endpoints; first occurrence numbers it
    e = np.stack([np.stack([a, b], 1), np.stack([b, c], 1), np.stack([c, a], 1)], 1).reshape(-1, 2)
    key = np.minimum(e[:, 0], e[:, 1]) * nv + np.maximum(e[:, 0], e[:, 1])
    uniq, first_idx, inv = np.unique(key, return_index=True, return_inverse=True)
    order = np.argsort(first_idx, kind="stable")          # number edges by first appearance
    rank = np.empty_like(order)
    rank[order] = np.arange(order.size)
    mid_id = nv + rank[inv]                                  # per (face, edge) new vertex id
    ue0 = e[first_idx[order], 0]
    ue1 = e[first_idx[order], 1]
    mpos = ((pos[ue0] + pos[ue1]) * np.float32(0.5)).astype(np.float32)
    mnrm = _normalize_rows((nrm[ue0] + nrm[ue1]).astype(np.float32))
    m = mid_id.reshape(-1, 3)
    ab, bc, ca = m[:, 0], m[:, 1], m[:, 2]
    nf = np.stack([
        np.stack([a, ab, ca], 1), np.stack([ab, b, bc], 1),
        np.stack([ca, bc, c], 1), np.stack([ab, bc, ca], 1)], 1).reshape(-1)
    return {
        "pos": np.concatenate([pos, mpos]).astype(np.float32),
        "nrm": np.concatenate([nrm, mnrm]).astype(np.float32),
        "idx": nf.astype(np.uint32),
    }


def scene(name: str):
    """Meshes of a named workload: bunny, suzanne, f16, armadillo_proxy, tyra_proxy, merged_proxy."""
    if name in ("bunny", "suzanne", "f16"):
        return load_mesh(name)
    bunny = load_mesh("bunny")[0]
    if name == "armadillo_proxy":
        return [subdivide(bunny)]
    if name == "tyra_proxy":
        return [subdivide(subdivide(bunny))]
    if name == "merged_proxy":
        return [subdivide(subdivide(bunny))] + load_mesh("f16")
    raise KeyError(name)


def sweep_views(n: int = 16, seed: int = 1234, radius: float = 3.5,
                center=(-0.337, 1.203, -0.031)):
    """Seeded eyes uniform on a sphere around the bunny, look-at orient as column-major mat3
    (columns = right, up, forward so that the reference's +z camera ray maps to forward)."""
    rng = np.random.default_rng(seed)
    v = rng.normal(size=(n, 3))
    v /= np.linalg.norm(v, axis=1, keepdims=True)
    c = np.asarray(center, np.float64)
    eyes = c + radius * v
    orients = []
    for e in eyes:
        fwd = c - e
        fwd /= np.linalg.norm(fwd)
        up0 = np.array([0.0, 1.0, 0.0]) if abs(fwd[1]) < 0.95 else np.array([1.0, 0.0, 0.0])
        right = np.cross(up0, fwd)
        right /= np.linalg.norm(right)
        up = np.cross(fwd, right)
        orients.append(np.concatenate([right, up, fwd]))  # column-major: m[0]=right, m[1]=up, m[2]=fwd
    return eyes.astype(np.float32), np.asarray(orients, np.float32)
