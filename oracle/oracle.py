"""ctypes binding of oracle/liboracle.so (test infrastructure only; see __init__.py)."""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "liboracle.so")


class _OrcMesh(C.Structure):
    _fields_ = [
        ("pos", C.POINTER(C.c_float)),
        ("nrm", C.POINTER(C.c_float)),
        ("idx", C.POINTER(C.c_uint32)),
        ("num_verts", C.c_uint32),
        ("num_idx", C.c_uint32),
    ]


class _OrcObj(C.Structure):
    _fields_ = [
        ("num_meshes", C.c_uint32),
        ("pos", C.POINTER(C.c_float) * 16),
        ("nrm", C.POINTER(C.c_float) * 16),
        ("idx", C.POINTER(C.c_uint32) * 16),
        ("num_verts", C.c_uint32 * 16),
        ("num_idx", C.c_uint32 * 16),
    ]


def build_oracle(force: bool = False) -> str:
    """Compile liboracle.so with the committed Makefile (gcc, IEEE, no contraction)."""
    src = os.path.join(_HERE, "beam_oracle.c")
    if force or not os.path.exists(_LIB) or os.path.getmtime(_LIB) < os.path.getmtime(src):
        subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB


_lib = None


def load_oracle() -> C.CDLL:
    global _lib
    if _lib is None:
        build_oracle()
        lib = C.CDLL(_LIB)
        f32p, u32p, u64p = C.POINTER(C.c_float), C.POINTER(C.c_uint32), C.POINTER(C.c_uint64)
        mp = C.POINTER(_OrcMesh)
        lib.orc_camera_rays.argtypes = [C.c_uint32, C.c_uint32] + [C.c_float] * 5 + [f32p]
        lib.orc_camera_rays.restype = C.c_int32
        lib.orc_kd_build.argtypes = [mp, C.c_uint32, C.c_float, C.c_float]
        lib.orc_kd_build.restype = C.c_void_p
        lib.orc_kd_stats.argtypes = [C.c_void_p, u64p]
        lib.orc_kd_free.argtypes = [C.c_void_p]
        lib.orc_kd_march.argtypes = [C.c_void_p, f32p, C.c_uint32, C.c_uint32, f32p, f32p, u32p, u32p, f32p]
        lib.orc_kd_march.restype = C.c_int32
        lib.orc_kd_march_counts.argtypes = [C.c_void_p, f32p, C.c_uint32, C.c_uint32, f32p, f32p, u64p]
        lib.orc_kd_march_counts.restype = C.c_int32
        lib.orc_hash_build.argtypes = [mp, C.c_uint32]
        lib.orc_hash_build.restype = C.c_void_p
        lib.orc_hash_free.argtypes = [C.c_void_p]
        lib.orc_hash_stats.argtypes = [C.c_void_p, u64p]
        lib.orc_hash_buckets.argtypes = [C.c_void_p, C.POINTER(u32p)]
        lib.orc_hash_buckets.restype = u32p
        lib.orc_hash_march.argtypes = [C.c_void_p, f32p, C.c_uint32, C.c_uint32, f32p, f32p, u32p, u32p, f32p]
        lib.orc_hash_march.restype = C.c_int32
        lib.orc_bvh_build.argtypes = [mp, C.c_uint32, C.c_uint32]
        lib.orc_bvh_build.restype = C.c_void_p
        lib.orc_bvh_build_ex.argtypes = [mp, C.c_uint32, C.c_uint32, C.c_uint32]
        lib.orc_bvh_build_ex.restype = C.c_void_p
        lib.orc_bvh_record_words.argtypes = [C.c_void_p]
        lib.orc_bvh_record_words.restype = C.c_uint32
        lib.orc_bvh_refit.argtypes = [C.c_void_p, mp, C.c_uint32]
        lib.orc_bvh_refit.restype = C.c_int32
        lib.orc_bvh_free.argtypes = [C.c_void_p]
        lib.orc_bvh_num_tris.argtypes = [C.c_void_p]
        lib.orc_bvh_num_tris.restype = C.c_uint32
        lib.orc_bvh_num_records.argtypes = [C.c_void_p]
        lib.orc_bvh_num_records.restype = C.c_uint32
        lib.orc_bvh_export.argtypes = [C.c_void_p, u32p, u32p, u32p, u32p]
        lib.orc_bvh_trace.argtypes = [C.c_void_p, f32p, C.c_uint32, C.c_uint32, f32p, f32p, u32p, u32p, f32p, u64p]
        lib.orc_bvh_trace.restype = C.c_int32
        lib.orc_brute_trace.argtypes = [mp, C.c_uint32, f32p, C.c_uint32, C.c_uint32, f32p, f32p, u32p, u32p, f32p]
        lib.orc_brute_trace.restype = C.c_int32
        u8p = C.POINTER(C.c_uint8)
        lib.orc_bvh_shadow.argtypes = [C.c_void_p, f32p, C.c_uint32, C.c_uint32, f32p, f32p, f32p, u32p, f32p, u8p,
                                       u64p]
        lib.orc_bvh_shadow.restype = C.c_int32
        lib.orc_brute_shadow.argtypes = [mp, C.c_uint32, f32p, C.c_uint32, C.c_uint32, f32p, f32p, f32p, u32p, f32p,
                                         u8p]
        lib.orc_brute_shadow.restype = C.c_int32
        lib.orc_obj_load.argtypes = [C.c_char_p, C.c_int32, C.POINTER(_OrcObj)]
        lib.orc_obj_load.restype = C.c_int32
        lib.orc_obj_free.argtypes = [C.POINTER(_OrcObj)]
        _lib = lib
    return _lib


def _p(a, ct):
    return a.ctypes.data_as(C.POINTER(ct)) if a is not None else None


class OrcMeshes:
    """Keeps numpy mesh arrays alive while the C side references them."""

    def __init__(self, meshes):
        self.meshes = []
        for m in meshes:
            pos = np.ascontiguousarray(m["pos"], dtype=np.float32).reshape(-1, 3)
            nrm = m.get("nrm")
            nrm = None if nrm is None else np.ascontiguousarray(nrm, dtype=np.float32).reshape(-1, 3)
            idx = np.ascontiguousarray(m["idx"], dtype=np.uint32).reshape(-1)
            self.meshes.append((pos, nrm, idx))
        self.arr = (_OrcMesh * max(1, len(self.meshes)))()
        for i, (pos, nrm, idx) in enumerate(self.meshes):
            self.arr[i] = _OrcMesh(_p(pos, C.c_float), _p(nrm, C.c_float), _p(idx, C.c_uint32), pos.shape[0], idx.size)

    @property
    def count(self):
        return len(self.meshes)

    @property
    def num_tris(self):
        return sum(m[2].size // 3 for m in self.meshes)


class Oracle:
    """Thin object API over liboracle.so."""

    def __init__(self):
        self.lib = load_oracle()

    # Camera::setInitialRays (Camera.cpp:43-72)
    def camera_rays(self, w, h, left=-1.0, right=1.0, top=1.0, bottom=-1.0, zoom=1.0):
        out = np.empty((h * w, 3), dtype=np.float32)
        err = self.lib.orc_camera_rays(w, h, left, right, top, bottom, zoom, _p(out, C.c_float))
        return err, out

    @staticmethod
    def _frame(n):
        return (np.empty(n, np.uint32), np.empty(n, np.uint32), np.empty(n, np.float32))

    # reference semantics
    def kd_render(self, meshes, rays, eye, orient, begin=0, end=None, wmin=-30.0, wmax=30.0, stats=False):
        om = meshes if isinstance(meshes, OrcMeshes) else OrcMeshes(meshes)
        n = rays.shape[0]
        end = n if end is None else end
        kd = self.lib.orc_kd_build(om.arr, om.count, wmin, wmax)
        try:
            st = np.zeros(8, np.uint64)
            self.lib.orc_kd_stats(kd, _p(st, C.c_uint64))
            packed, tri, t = self._frame(n)
            eye = np.asarray(eye, np.float32)
            orient = np.asarray(orient, np.float32).reshape(9)
            rays = np.ascontiguousarray(rays, np.float32)
            err = self.lib.orc_kd_march(kd, _p(rays, C.c_float), begin, end, _p(eye, C.c_float),
                                        _p(orient, C.c_float), _p(packed, C.c_uint32), _p(tri, C.c_uint32),
                                        _p(t, C.c_float))
        finally:
            self.lib.orc_kd_free(kd)
        if err:
            raise RuntimeError(f"orc_kd_march error {err}")
        res = (packed[begin:end], tri[begin:end], t[begin:end])
        return (res + (st,)) if stats else res

    def kd_build(self, meshes, wmin=-30.0, wmax=30.0):
        """The reference's kd-tree (orc_kd_build), kept for repeated marches (CPU baseline)."""
        om = meshes if isinstance(meshes, OrcMeshes) else OrcMeshes(meshes)
        return OrcKd(self.lib, om, wmin, wmax)

    # reference semantics, alternative accelerator: hashed uniform grid (Hash.cu, insert loop fixed)
    def hash_render(self, meshes, rays, eye, orient, begin=0, end=None, stats=False, buckets=False):
        om = meshes if isinstance(meshes, OrcMeshes) else OrcMeshes(meshes)
        n = rays.shape[0]
        end = n if end is None else end
        hg = self.lib.orc_hash_build(om.arr, om.count)
        if not hg:
            raise RuntimeError("orc_hash_build: a triangle spans more than 2^20 cells")
        try:
            st = np.zeros(4, np.uint64)
            self.lib.orc_hash_stats(hg, _p(st, C.c_uint64))
            bk = None
            if buckets:
                fp = C.POINTER(C.c_uint32)()
                sp = self.lib.orc_hash_buckets(hg, C.byref(fp))
                start = np.ctypeslib.as_array(sp, shape=(65537,)).copy()
                faces = np.ctypeslib.as_array(fp, shape=(max(1, int(start[-1])),))[:int(start[-1])].copy()
                bk = (start, faces)
            packed, tri, t = self._frame(n)
            eye = np.asarray(eye, np.float32)
            orient = np.asarray(orient, np.float32).reshape(9)
            rays = np.ascontiguousarray(rays, np.float32)
            err = self.lib.orc_hash_march(hg, _p(rays, C.c_float), begin, end, _p(eye, C.c_float),
                                          _p(orient, C.c_float), _p(packed, C.c_uint32), _p(tri, C.c_uint32),
                                          _p(t, C.c_float))
        finally:
            self.lib.orc_hash_free(hg)
        if err:
            raise RuntimeError(f"orc_hash_march error {err}")
        res = (packed[begin:end], tri[begin:end], t[begin:end])
        if stats:
            res = res + (st,)
        if buckets:
            res = res + (bk,)
        return res

    def bvh_build(self, meshes, leaf_size=4, width=2):
        om = meshes if isinstance(meshes, OrcMeshes) else OrcMeshes(meshes)
        return OrcBVH(self.lib, om, leaf_size, width)

    def brute_render(self, meshes, rays, eye, orient, begin=0, end=None):
        om = meshes if isinstance(meshes, OrcMeshes) else OrcMeshes(meshes)
        n = rays.shape[0]
        end = n if end is None else end
        packed, tri, t = self._frame(n)
        eye = np.asarray(eye, np.float32)
        orient = np.asarray(orient, np.float32).reshape(9)
        rays = np.ascontiguousarray(rays, np.float32)
        err = self.lib.orc_brute_trace(om.arr, om.count, _p(rays, C.c_float), begin, end, _p(eye, C.c_float),
                                       _p(orient, C.c_float), _p(packed, C.c_uint32), _p(tri, C.c_uint32),
                                       _p(t, C.c_float))
        if err:
            raise RuntimeError(f"orc_brute_trace error {err}")
        return packed[begin:end], tri[begin:end], t[begin:end]

    def brute_shadow(self, meshes, rays, eye, orient, light, tri, t):
        """Exhaustive any-hit shadow rays for a primary frame (tri, t indexed like rays)."""
        om = meshes if isinstance(meshes, OrcMeshes) else OrcMeshes(meshes)
        n = rays.shape[0]
        out = np.zeros(n, np.uint8)
        a = _shadow_args(rays, eye, orient, light, tri, t)
        err = self.lib.orc_brute_shadow(om.arr, om.count, _p(a[0], C.c_float), 0, n, _p(a[1], C.c_float),
                                        _p(a[2], C.c_float), _p(a[3], C.c_float), _p(a[4], C.c_uint32),
                                        _p(a[5], C.c_float), _p(out, C.c_uint8))
        if err:
            raise RuntimeError(f"orc_brute_shadow error {err}")
        return out

    def load_obj(self, path, share=1):
        o = _OrcObj()
        nm = self.lib.orc_obj_load(path.encode(), int(share), C.byref(o))
        if nm < 0:
            raise FileNotFoundError(path)
        meshes = []
        for m in range(nm):
            nv, ni = o.num_verts[m], o.num_idx[m]
            pos = np.ctypeslib.as_array(o.pos[m], shape=(nv * 3,)).reshape(nv, 3).copy()
            nrm = None
            if o.nrm[m]:
                nrm = np.ctypeslib.as_array(o.nrm[m], shape=(nv * 3,)).reshape(nv, 3).copy()
            idx = np.ctypeslib.as_array(o.idx[m], shape=(ni,)).copy()
            meshes.append({"pos": pos, "nrm": nrm, "idx": idx})
        self.lib.orc_obj_free(C.byref(o))
        return meshes


def _shadow_args(rays, eye, orient, light, tri, t):
    return (np.ascontiguousarray(rays, np.float32), np.asarray(eye, np.float32),
            np.asarray(orient, np.float32).reshape(9), np.asarray(light, np.float32),
            np.ascontiguousarray(tri, np.uint32).reshape(-1), np.ascontiguousarray(t, np.float32).reshape(-1))


class OrcKd:
    """orc_kd_build once, orc_kd_march over pixel ranges (ctypes releases the GIL: threads run in
    parallel), freed with the object."""

    def __init__(self, lib, om, wmin, wmax):
        self.lib, self.om = lib, om
        self.h = lib.orc_kd_build(om.arr, om.count, wmin, wmax)

    def __del__(self):
        if getattr(self, "h", None):
            self.lib.orc_kd_free(self.h)
            self.h = None

    def render(self, rays, eye, orient, begin=0, end=None):
        n = rays.shape[0]
        end = n if end is None else end
        packed, tri, t = Oracle._frame(n)
        eye = np.asarray(eye, np.float32)
        orient = np.asarray(orient, np.float32).reshape(9)
        err = self.lib.orc_kd_march(self.h, _p(rays, C.c_float), begin, end, _p(eye, C.c_float),
                                    _p(orient, C.c_float), _p(packed, C.c_uint32), _p(tri, C.c_uint32),
                                    _p(t, C.c_float))
        if err:
            raise RuntimeError(f"orc_kd_march error {err}")
        return packed[begin:end], tri[begin:end], t[begin:end]

    def counts(self, rays, eye, orient, begin=0, end=None):
        """(node pops = box tests, leaves entered, face tests) of the march over [begin, end)."""
        n = rays.shape[0]
        end = n if end is None else end
        out = np.zeros(3, np.uint64)
        eye = np.asarray(eye, np.float32)
        orient = np.asarray(orient, np.float32).reshape(9)
        self.lib.orc_kd_march_counts(self.h, _p(rays, C.c_float), begin, end, _p(eye, C.c_float),
                                     _p(orient, C.c_float), _p(out, C.c_uint64))
        return out


class OrcBVH:
    def __init__(self, lib, om, leaf_size, width=2):
        self.lib, self.om = lib, om
        self.h = lib.orc_bvh_build_ex(om.arr, om.count, leaf_size, width)
        self.width = width
        self.record_words = lib.orc_bvh_record_words(self.h)
        self.n = lib.orc_bvh_num_tris(self.h)
        self.num_records = lib.orc_bvh_num_records(self.h)

    def __del__(self):
        if getattr(self, "h", None):
            self.lib.orc_bvh_free(self.h)
            self.h = None

    def refit(self, meshes):
        """Same topology, new vertex data (orc_bvh_refit); meshes must keep the triangle count."""
        om = meshes if isinstance(meshes, OrcMeshes) else OrcMeshes(meshes)
        err = self.lib.orc_bvh_refit(self.h, om.arr, om.count)
        if err:
            raise ValueError(f"orc_bvh_refit error {err}")
        self.om = om
        return self

    def export(self):
        rec = np.zeros((self.num_records, self.record_words), np.uint32)
        tris = np.zeros((max(self.n, 1), 12), np.uint32)
        keys = np.zeros(max(self.n, 1), np.uint32)
        perm = np.zeros(max(self.n, 1), np.uint32)
        self.lib.orc_bvh_export(self.h, _p(rec, C.c_uint32), _p(tris, C.c_uint32), _p(keys, C.c_uint32),
                                _p(perm, C.c_uint32))
        return rec, tris[: self.n], keys[: self.n], perm[: self.n]

    def render(self, rays, eye, orient, begin=0, end=None, counters=False):
        n = rays.shape[0]
        end = n if end is None else end
        packed, tri, t = Oracle._frame(n)
        cnt = np.zeros(3, np.uint64)
        eye = np.asarray(eye, np.float32)
        orient = np.asarray(orient, np.float32).reshape(9)
        rays = np.ascontiguousarray(rays, np.float32)
        err = self.lib.orc_bvh_trace(self.h, _p(rays, C.c_float), begin, end, _p(eye, C.c_float),
                                     _p(orient, C.c_float), _p(packed, C.c_uint32), _p(tri, C.c_uint32),
                                     _p(t, C.c_float), _p(cnt, C.c_uint64))
        if err:
            raise RuntimeError(f"orc_bvh_trace error {err}")
        res = (packed[begin:end], tri[begin:end], t[begin:end])
        return (res + (cnt,)) if counters else res

    def shadow(self, rays, eye, orient, light, tri, t, counters=False):
        """One any-hit shadow ray per primary hit (orc_bvh_shadow); returns u8 per pixel."""
        n = rays.shape[0]
        out = np.zeros(n, np.uint8)
        cnt = np.zeros(3, np.uint64)
        a = _shadow_args(rays, eye, orient, light, tri, t)
        err = self.lib.orc_bvh_shadow(self.h, _p(a[0], C.c_float), 0, n, _p(a[1], C.c_float), _p(a[2], C.c_float),
                                      _p(a[3], C.c_float), _p(a[4], C.c_uint32), _p(a[5], C.c_float),
                                      _p(out, C.c_uint8), _p(cnt, C.c_uint64))
        if err:
            raise RuntimeError(f"orc_bvh_shadow error {err}")
        return (out, cnt) if counters else out
