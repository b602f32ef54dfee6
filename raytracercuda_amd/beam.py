"""Python mirror of the reference's Beam host API (Raytracer/Beam.h:32-72) over the C ABI.

Same class and method names, argument meaning and u32 error codes as the reference:

    ctx    = Context(device=0)                       # new: explicit device/stream context
    mesh   = IMesh.create(ctx)
    mesh.setIndices(idx, len(idx)); mesh.setVertexData(pos, nv, 3, VERTEX_DATA_POSITION)
    scene  = IScene.create(ctx); scene.addMesh(mesh); scene.updateGPUScene()
    cam    = ICamera.create(ctx); cam.setInitialRays(W, H, -1, 1, -1, 1, 1)
    rt     = IRenderTarget.createOffscreen(ctx, W, H)   # replaces registerGLTBO
    rt.lock(); cam.traceScene(eye3, orient3x3, scene); rt.unlock()

As in the reference (RenderTarget.cpp:53-88), lock() makes the target the process-wide current
render target that traceScene()/clear() use. Device work is asynchronous on the context stream;
ctx.sync() or a read waits.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from . import _lib
from ._lib import (ERROR_ALL_FINE, ERROR_DEVICE, ERROR_GPU_ALLOC_FAIL, ERROR_INVALID_FORMAT,  # noqa: F401
                   ERROR_INVALID_PARAMETER, ERROR_LOCK_FIRST, ERROR_NO_RENDER_TARGET, ERROR_NO_VERTICES,
                   ERROR_NOT_BUILT, ERROR_RT_CAM_MISMATCH, ERROR_UNLOCK_FIRST, MISS_PACKED, NO_TRIANGLE,
                   VERTEX_DATA_COUNT, VERTEX_DATA_NORMAL, VERTEX_DATA_POSITION, BeamError, BuildStats, Options,
                   SORT_LSD, SORT_MSD, SORT_MSD_SKEW, SORT_KD_RANKED)


def _f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


def _fp(a):
    return a.ctypes.data_as(C.POINTER(C.c_float))


def _up(a):
    return a.ctypes.data_as(C.POINTER(C.c_uint32))


def comm_unique_id() -> bytes:
    """Rank 0 of a multi-process context makes the RCCL unique id every rank passes as comm_id."""
    lib = _lib.load()
    buf = (C.c_uint8 * _lib.COMM_ID_BYTES)()
    err = lib.bm_comm_unique_id(buf)
    if err:
        raise BeamError(err, "bm_comm_unique_id: RCCL unavailable")
    return bytes(buf)


def ab_build() -> bool:
    """Whether the loaded library is an A/B build (tools/build_ab.py ... BM_TRACE_AB=1): the trace
    variants measured slower than the product kernels and BVH8 are compiled in (bm_version "+ab")."""
    return _lib.load().bm_version().decode().endswith("+ab")


def comm_available() -> None:
    """Raises BeamError unless RCCL resolves in this process (bm_comm_available): what every rank
    checks before any rank starts the communicator (multigpu.start_comm)."""
    err = _lib.load().bm_comm_available()
    if err:
        raise BeamError(err, "bm_comm_available: RCCL (librccl.so.1) unavailable")


_GATHER = {"auto": _lib.GATHER_AUTO, "peer": _lib.GATHER_PEER, "rccl": _lib.GATHER_RCCL}
_PLANES = {"packed": _lib.PLANE_PACKED, "tri_id": _lib.PLANE_TRI_ID, "t": _lib.PLANE_T, "nz": _lib.PLANE_NZ,
           "shadow": _lib.PLANE_SHADOW}


class Context:
    """One device + one HIP stream (bm_context), or a multi-GPU context:

    * devices=[d0, d1, ...] (one process): objects are replicated on every listed device and a trace
      deals 16-row screen bands round-robin to them, gathered into the render target on d0
      (gather "peer": xGMI writes from each device; "rccl": one RCCL communicator). Repeating a device
      rehearses the n-way path on one GPU.
    * comm=(rank, size, unique_id) (one process per GPU): this rank's bands, gathered into rank 0's
      render target over RCCL.
    planes: which planes the gather carries ("packed", "tri_id", "t", "nz", "shadow"; None = all).
    params: tuning parameters {name: value} (bm_context_set_param; names in _lib.PARAMS), set right
    after creation: measurement and test hooks, the defaults being the measured-best schedules."""

    def __init__(self, device: int = 0, stream: int | None = None, leaf_size: int = 4, shadow_queue: bool = False,
                 bvh_width: int = 4, reference_kd: bool = False, reference_hash: bool = False, devices=None,
                 band_height: int = 0, gather: str = "auto", planes=None, comm=None, params=None):
        self.lib = _lib.load()
        h = C.c_void_p()
        # stream=None: the context owns a stream; an int (0 = the null stream) is used as given
        flags = _lib.OPT_NULL_STREAM if stream == 0 else 0
        if shadow_queue:  # shadow rays as a separate wavefront pass (compaction study)
            flags |= _lib.OPT_SHADOW_QUEUE
        if bvh_width == 2:  # binary BVH (64-B records) instead of BVH4
            flags |= _lib.OPT_BVH2
        if bvh_width == 8:  # BVH8 (256-B records, three binary levels per node; quad kernel only)
            flags |= _lib.OPT_BVH8
        if reference_kd:  # the reference's own kd-tree + march: frames equal to the reference's
            flags |= _lib.OPT_REFERENCE_KD
        if reference_hash:  # the reference's hashed uniform grid (Hash.cu) + its cell march
            flags |= _lib.OPT_REFERENCE_HASH
        opts = Options(device, C.c_void_p(stream) if stream else None, leaf_size, flags)
        if devices:
            devices = list(devices)
            if len(devices) > _lib.MAX_DEVICES:
                raise BeamError(ERROR_INVALID_PARAMETER, f"at most {_lib.MAX_DEVICES} devices")
            opts.num_devices = len(devices)
            for i, d in enumerate(devices):
                opts.devices[i] = d
            device = devices[0]
        opts.band_height = band_height
        opts.gather = _GATHER[gather]
        opts.gather_planes = sum(_PLANES[p] for p in planes) if planes else 0
        if comm is not None:
            rank, size, uid = comm
            opts.comm_rank, opts.comm_size = rank, size
            C.memmove(opts.comm_id, bytes(uid), _lib.COMM_ID_BYTES)
        err = self.lib.bm_context_create(C.byref(opts), C.byref(h))
        if err:
            raise BeamError(err, f"bm_context_create(device={device}, devices={devices}, comm="
                                 f"{None if comm is None else comm[:2]}) failed")
        self.h = h
        self.device = device
        self.num_devices = int(self.lib.bm_context_num_devices(h))
        # the transport the library resolved: "peer", "rccl", "rccl-loopback" (a repeated device
        # list over one single-rank communicator) or None (one device)
        self.gather = {1: "peer", 2: "rccl", 3: "rccl-loopback"}.get(int(self.lib.bm_context_gather(h)))
        self.bvh_width = bvh_width if bvh_width in (2, 8) else 4
        for k, v in (params or {}).items():
            self.set_param(k, v)

    def set_param(self, name: str, value: int) -> None:
        """bm_context_set_param by name (_lib.PARAMS); -1 restores the library default."""
        if name not in _lib.PARAMS:
            raise BeamError(ERROR_INVALID_PARAMETER, f"unknown parameter {name!r}")
        self._check(self.lib.bm_context_set_param(self.h, _lib.PARAMS[name], int(value)))

    def get_param(self, name: str) -> int:
        """The value set for a parameter, -1 while the library default is in effect."""
        return int(self.lib.bm_context_get_param(self.h, _lib.PARAMS[name]))

    def start_comm(self, rank: int, size: int, unique_id: bytes) -> None:
        """Join the multi-process RCCL communicator (bm_context_start_comm) on a context created
        without one: the collective ncclCommInitRank, entered only after every rank's device context
        exists (multigpu.start_comm)."""
        uid = (C.c_uint8 * _lib.COMM_ID_BYTES).from_buffer_copy(bytes(unique_id)[:_lib.COMM_ID_BYTES])
        self._check(self.lib.bm_context_start_comm(self.h, rank, size, uid))
        self.num_devices = int(self.lib.bm_context_num_devices(self.h))
        self.gather = {1: "peer", 2: "rccl", 3: "rccl-loopback"}.get(int(self.lib.bm_context_gather(self.h)))

    def sync(self):
        self._check(self.lib.bm_sync(self.h))

    def debug_primitives(self, records):
        """bm_debug_primitives: the trace kernels' scalar primitives on float32 records [n, 36] ->
        [n, 12] (layouts in include/beam_c.h; tests/test_gpu_glm_pin.py)."""
        inp = np.ascontiguousarray(records, np.float32).reshape(-1, 36)
        out = np.zeros((inp.shape[0], 12), np.float32)
        self._check(self.lib.bm_debug_primitives(self.h, inp.shape[0], inp.ctypes.data, out.ctypes.data))
        return out

    @property
    def stream(self) -> int:
        return self.lib.bm_context_stream(self.h) or 0

    def last_error(self) -> str:
        return (self.lib.bm_last_error_string(self.h) or b"").decode()

    def _check(self, err):
        if err:
            raise BeamError(err, self.last_error())
        return err

    def close(self):
        if getattr(self, "h", None):
            self.lib.bm_context_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass


class IMesh:
    """Raytracer/Beam.h:47-54, Mesh.cpp."""

    def __init__(self, ctx: Context):
        self.ctx = ctx
        h = C.c_void_p()
        ctx._check(ctx.lib.bm_mesh_create(ctx.h, C.byref(h)))
        self.h = h

    @staticmethod
    def create(ctx: Context) -> "IMesh":
        return IMesh(ctx)

    def setVertexData(self, vertices, numVertices: int, numComponents: int, slotId: int, asyncCopy: bool = False):
        a = _f32(vertices).reshape(-1)
        if a.size < numVertices * numComponents:
            return ERROR_INVALID_PARAMETER
        return self.ctx.lib.bm_mesh_set_vertex_data(self.h, _fp(a), numVertices, numComponents, slotId)

    def setIndices(self, indices, numIndices: int, asyncCopy: bool = False):
        a = np.ascontiguousarray(indices, dtype=np.uint32).reshape(-1)
        if a.size < numIndices:
            return ERROR_INVALID_PARAMETER
        return self.ctx.lib.bm_mesh_set_indices(self.h, _up(a), numIndices)

    def destroy(self):
        if getattr(self, "h", None) and self.ctx.h:
            self.ctx.lib.bm_mesh_destroy(self.h)
        self.h = None


class IScene:
    """Raytracer/Beam.h:56-63, Scene.cpp / SceneTree.cpp (acceleration structure = LBVH)."""

    def __init__(self, ctx: Context):
        self.ctx = ctx
        h = C.c_void_p()
        ctx._check(ctx.lib.bm_scene_create(ctx.h, C.byref(h)))
        self.h = h
        self.meshes = []  # keep meshes alive (sptr semantics)
        self.last_stats = None

    @staticmethod
    def create(ctx: Context) -> "IScene":
        return IScene(ctx)

    def addMesh(self, mesh: IMesh):
        self.ctx._check(self.ctx.lib.bm_scene_add_mesh(self.h, mesh.h))
        self.meshes.append(mesh)

    def removeMesh(self, mesh: IMesh):
        self.ctx._check(self.ctx.lib.bm_scene_remove_mesh(self.h, mesh.h))
        self.meshes = [m for m in self.meshes if m is not mesh]

    def updateGPUScene(self, stats: bool = False):
        """Rebuild the BVH from the current meshes (asynchronous unless stats=True)."""
        st = BuildStats()
        self.ctx._check(self.ctx.lib.bm_scene_build(self.h, C.byref(st) if stats else None))
        if stats:
            self.last_stats = {f: getattr(st, f) for f, _ in BuildStats._fields_}
            return self.last_stats
        return None

    def kdStats(self):
        """Reference mode: [leaves with faces, face refs stored, faces dropped (cap 256), largest leaf]."""
        out = np.zeros(4, np.uint64)
        self.ctx._check(self.ctx.lib.bm_scene_kd_stats(self.h, out.ctypes.data_as(C.POINTER(C.c_uint64))))
        return out

    def gridStats(self):
        """Hashed-grid mode: [(cell, face) pairs, non-empty buckets, largest bucket, faces beyond
        the 256 cap]."""
        out = np.zeros(4, np.uint64)
        self.ctx._check(self.ctx.lib.bm_scene_grid_stats(self.h, out.ctypes.data_as(C.POINTER(C.c_uint64))))
        return out

    def gridExport(self):
        """Hashed-grid mode: (bucket_start[65536], bucket_end[65536], faces[pairs])."""
        pairs = int(self.gridStats()[0])
        b0 = np.zeros(65536, np.uint32)
        b1 = np.zeros(65536, np.uint32)
        faces = np.zeros(max(1, pairs), np.uint32)
        u32 = C.POINTER(C.c_uint32)
        self.ctx._check(self.ctx.lib.bm_scene_grid_export(self.h, b0.ctypes.data_as(u32), b1.ctypes.data_as(u32),
                                                          faces.ctypes.data_as(u32)))
        return b0, b1, faces[:pairs]

    def refitGPUScene(self, stats: bool = False):
        """Refit-only update after vertex data changed (bm_scene_refit): same meshes and triangle
        counts as the last updateGPUScene; raises BeamError otherwise."""
        st = BuildStats()
        self.ctx._check(self.ctx.lib.bm_scene_refit(self.h, C.byref(st) if stats else None))
        if stats:
            self.last_stats = {f: getattr(st, f) for f, _ in BuildStats._fields_}
            return self.last_stats
        return None

    def export(self):
        """(records[nrec, 16, 32 or 64], tris[n,12], keys[n], perm[n]) as uint32 — for parity tests.
        BVH4 records are written for every node above the leaf size, but a traversal reaches only
        the even-depth ones (the others are expanded into their parents' records) and the oracle
        writes only those: compare reachable_records rather than the whole array."""
        st = self.last_stats or self.updateGPUScene(stats=True)
        n, nrec = st["num_tris"], st["num_records"]
        rec = np.zeros((nrec, {8: 64, 4: 32}.get(st["bvh_width"], 16)), np.uint32)
        tris = np.zeros((max(n, 1), 12), np.uint32)
        keys = np.zeros(max(n, 1), np.uint32)
        perm = np.zeros(max(n, 1), np.uint32)
        self.ctx._check(self.ctx.lib.bm_scene_export(self.h, _up(rec), _up(tris), _up(keys), _up(perm)))
        return rec, tris[:n], keys[:n], perm[:n]

    def destroy(self):
        if getattr(self, "h", None) and self.ctx.h:
            self.ctx.lib.bm_scene_destroy(self.h)
        self.h = None


class IRenderTarget:
    """Raytracer/Beam.h:32-45 with an offscreen device buffer instead of a GL TBO."""

    _current = None  # RenderTarget::m_RT (RenderTarget.cpp:85-93)

    def __init__(self, ctx: Context, handle, keepalive=None):
        self.ctx = ctx
        self.h = handle
        self._keep = keepalive
        self._locked = False

    @staticmethod
    def createOffscreen(ctx: Context, width: int, height: int, pitch: int = 0) -> "IRenderTarget":
        h = C.c_void_p()
        ctx._check(ctx.lib.bm_rt_create_offscreen(ctx.h, width, height, pitch, C.byref(h)))
        return IRenderTarget(ctx, h)

    @staticmethod
    def createExternal(ctx: Context, width: int, height: int, pitch: int, packed_ptr: int, tri_ptr: int,
                       t_ptr: int, nz_ptr: int = 0, keepalive=None) -> "IRenderTarget":
        h = C.c_void_p()
        ctx._check(ctx.lib.bm_rt_create_external(ctx.h, width, height, pitch, C.c_void_p(packed_ptr),
                                                 C.c_void_p(tri_ptr), C.c_void_p(t_ptr),
                                                 C.c_void_p(nz_ptr) if nz_ptr else None, C.byref(h)))
        return IRenderTarget(ctx, h, keepalive)

    def buffer(self) -> int:
        return self.ctx.lib.bm_rt_buffer(self.h) or 0

    def width(self) -> int:
        return self.ctx.lib.bm_rt_width(self.h)

    def height(self) -> int:
        return self.ctx.lib.bm_rt_height(self.h)

    def pitch(self) -> int:
        return self.ctx.lib.bm_rt_pitch(self.h)

    def lock(self) -> int:
        err = self.ctx.lib.bm_rt_lock(self.h)
        if err == ERROR_ALL_FINE:
            IRenderTarget._current = self
        return err

    def unlock(self) -> int:
        err = self.ctx.lib.bm_rt_unlock(self.h)
        if err == ERROR_ALL_FINE and IRenderTarget._current is self:
            IRenderTarget._current = None
        return err

    @staticmethod
    def get():
        return IRenderTarget._current

    def read(self, packed=True, tri_id=True, t=True, rgb=False):
        """Synchronous readback -> dict of (H, W) numpy planes (rgb: (H, W, 3))."""
        w, h = self.width(), self.height()
        out = {}
        bufs = {}
        if packed:
            bufs["packed"] = np.empty((h, w), np.uint32)
        if tri_id:
            bufs["tri_id"] = np.empty((h, w), np.uint32)
        if t:
            bufs["t"] = np.empty((h, w), np.float32)
        if rgb:
            bufs["rgb"] = np.empty((h, w, 3), np.float32)
        self.ctx._check(self.ctx.lib.bm_rt_read(
            self.h, _up(bufs["packed"]) if packed else None, _up(bufs["tri_id"]) if tri_id else None,
            _fp(bufs["t"]) if t else None, _fp(bufs["rgb"]) if rgb else None))
        out.update(bufs)
        return out

    def setStream(self, stream) -> None:
        """Frames in flight: this target's traces and readbacks on its own HIP stream (an int handle,
        e.g. torch.cuda.Stream().cuda_stream; None or 0: the context stream). See bm_rt_set_stream."""
        self.ctx._check(self.ctx.lib.bm_rt_set_stream(self.h, C.c_void_p(stream) if stream else None))

    def stream(self) -> int:
        """Handle of the stream this target's work runs on."""
        return self.ctx.lib.bm_rt_stream(self.h) or 0

    TRACE_KINDS = {0: "quads", 1: "cull+quads", 2: "lanes", 3: "kd march", 4: "hash march", 5: "packets"}

    def traceKind(self) -> str:
        """Kernels the last trace into this target ran (bm_rt_trace_kind): quads, cull+quads, ..."""
        return self.TRACE_KINDS.get(int(self.ctx.lib.bm_rt_trace_kind(self.h)), "none")

    def lastTiming(self):
        """Multi-device contexts: (band trace ms, exchange ms) of the last frame traced into this
        target, from HIP events (bm_rt_last_timing; waits for that frame)."""
        out = (C.c_float * 2)()
        self.ctx._check(self.ctx.lib.bm_rt_last_timing(self.h, out))
        return float(out[0]), float(out[1])

    def savePPM(self, path) -> None:
        """Binary PPM (P6) of the packed plane, written by the library (bm_rt_save_ppm)."""
        self.ctx._check(self.ctx.lib.bm_rt_save_ppm(self.h, os.fsencode(path)))

    def shadow(self) -> int:
        """Device pointer of the u8 shadow plane (0 before the first shadow trace)."""
        return self.ctx.lib.bm_rt_shadow(self.h) or 0

    def readShadow(self):
        """Synchronous readback of the shadow plane -> (H, W) uint8 (1 = shadowed)."""
        out = np.empty((self.height(), self.width()), np.uint8)
        self.ctx._check(self.ctx.lib.bm_rt_read_shadow(self.h, out.ctypes.data_as(C.POINTER(C.c_uint8))))
        return out

    def destroy(self):
        if getattr(self, "h", None) and self.ctx.h:
            if IRenderTarget._current is self:
                IRenderTarget._current = None
            self.ctx.lib.bm_rt_destroy(self.h)
        self.h = None


class ICamera:
    """Raytracer/Beam.h:65-72, Camera.cpp."""

    def __init__(self, ctx: Context):
        self.ctx = ctx
        h = C.c_void_p()
        ctx._check(ctx.lib.bm_camera_create(ctx.h, C.byref(h)))
        self.h = h

    @staticmethod
    def create(ctx: Context) -> "ICamera":
        return ICamera(ctx)

    def setInitialRays(self, width, height, left=-1.0, right=1.0, top=1.0, bottom=-1.0, zoom=1.0) -> int:
        return self.ctx.lib.bm_camera_set_initial_rays(self.h, width, height, left, right, top, bottom, zoom)

    def clear(self, value: int) -> int:
        rt = IRenderTarget.get()
        if rt is None:
            return ERROR_NO_RENDER_TARGET
        return self.ctx.lib.bm_rt_clear(rt.h, value)

    @staticmethod
    def _eo(eye3, orient3x3):
        e = _f32(eye3).reshape(3)
        o = _f32(orient3x3).reshape(9)
        return e, o

    def traceScene(self, eye3, orient3x3, scene: IScene) -> int:
        rt = IRenderTarget.get()
        if rt is None:
            return ERROR_NO_RENDER_TARGET
        return self.trace(eye3, orient3x3, scene, rt)

    def trace(self, eye3, orient3x3, scene: IScene, rt: IRenderTarget) -> int:
        e, o = self._eo(eye3, orient3x3)
        return self.ctx.lib.bm_camera_trace(self.h, _fp(e), _fp(o), scene.h, rt.h)

    def traceBands(self, eye3, orient3x3, scene: IScene, rt: IRenderTarget, band_height: int, band_step: int,
                   band_first: int) -> int:
        e, o = self._eo(eye3, orient3x3)
        return self.ctx.lib.bm_camera_trace_bands(self.h, _fp(e), _fp(o), scene.h, rt.h, band_height, band_step,
                                                  band_first)

    def traceShadow(self, eye3, orient3x3, scene: IScene, rt: IRenderTarget, light3) -> int:
        """Primary trace + one any-hit shadow ray per hit toward the point light light3."""
        e, o = self._eo(eye3, orient3x3)
        lt = _f32(light3).reshape(3)
        return self.ctx.lib.bm_camera_trace_shadow(self.h, _fp(e), _fp(o), scene.h, rt.h, _fp(lt))

    def traceShadowBands(self, eye3, orient3x3, scene: IScene, rt: IRenderTarget, band_height: int,
                         band_step: int, band_first: int, light3) -> int:
        e, o = self._eo(eye3, orient3x3)
        lt = _f32(light3).reshape(3)
        return self.ctx.lib.bm_camera_trace_shadow_bands(self.h, _fp(e), _fp(o), scene.h, rt.h, band_height,
                                                         band_step, band_first, _fp(lt))

    def traceShadowCounters(self, eye3, orient3x3, scene: IScene, rt: IRenderTarget, light3):
        """[primary nodes, tris, hits, shadow nodes, shadow tris, shadowed pixels]."""
        e, o = self._eo(eye3, orient3x3)
        lt = _f32(light3).reshape(3)
        out = np.zeros(6, np.uint64)
        self.ctx._check(self.ctx.lib.bm_camera_trace_shadow_counters(
            self.h, _fp(e), _fp(o), scene.h, rt.h, _fp(lt), out.ctypes.data_as(C.POINTER(C.c_uint64))))
        return out

    def traceCounters(self, eye3, orient3x3, scene: IScene, rt: IRenderTarget):
        e, o = self._eo(eye3, orient3x3)
        out = np.zeros(3, np.uint64)
        self.ctx._check(self.ctx.lib.bm_camera_trace_counters(
            self.h, _fp(e), _fp(o), scene.h, rt.h, out.ctypes.data_as(C.POINTER(C.c_uint64))))
        return out

    def traceProfile(self, eye3, orient3x3, scene: IScene, rt: IRenderTarget):
        """Diagnostic trace: per-wave (start, end, placement, work) as a uint64 [waves, 4] array."""
        e, o = self._eo(eye3, orient3x3)
        n = C.c_uint32(0)
        self.ctx.lib.bm_camera_trace_profile(self.h, _fp(e), _fp(o), scene.h, rt.h, None, 0, C.byref(n))
        cap = n.value
        out = np.zeros((cap, 4), np.uint64)
        self.ctx._check(self.ctx.lib.bm_camera_trace_profile(
            self.h, _fp(e), _fp(o), scene.h, rt.h, out.ctypes.data_as(C.POINTER(C.c_uint64)), cap, C.byref(n)))
        return out[: n.value]

    def destroy(self):
        if getattr(self, "h", None) and self.ctx.h:
            self.ctx.lib.bm_camera_destroy(self.h)
        self.h = None


class Model:
    """TestProgram/Model.cpp Model::load over the native OBJ reader (bm_model_*, csrc/bm_obj.cpp)."""

    def __init__(self, path: str, unshared: bool = False):
        self.lib = _lib.load()
        h = C.c_void_p()
        err = self.lib.bm_model_load(os.fsencode(path), _lib.OBJ_UNSHARED if unshared else 0, C.byref(h))
        if err:
            raise BeamError(err, f"bm_model_load({path!r}) failed")
        self.h = h
        self.ctx = None

    @staticmethod
    def load(ctx: "Context", name: str, toScene: "IScene", numAdds: int = 1) -> "Model":
        """Model::load(name, toScene, numAdds): parse, create one IMesh per mesh, add each numAdds times."""
        m = Model(name)
        m.upload(ctx, toScene, numAdds)
        return m

    def info(self) -> dict:
        st = _lib.ModelInfo()
        self.lib.bm_model_info_get(self.h, C.byref(st))
        return {"num_meshes": st.num_meshes, "num_faces": st.num_faces, "num_vertices": st.num_vertices,
                "bmin": list(st.bmin), "bmax": list(st.bmax)}

    def meshes(self):
        """Parsed meshes as dicts {pos (V,3), nrm (V,3) or None, uv (V,2) or None, tan / bit (V,3) or None
        (tangent space, meshes with normals and UVs), idx (3F,), material}."""
        out = []
        for i in range(self.info()["num_meshes"]):
            pos, nrm, uv = _FPtr(), _FPtr(), _FPtr()
            idx = C.POINTER(C.c_uint32)()
            nv, ni = C.c_uint32(), C.c_uint32()
            mat = C.c_char_p()
            self.lib.bm_model_mesh(self.h, i, C.byref(pos), C.byref(nrm), C.byref(uv), C.byref(idx), C.byref(nv),
                                   C.byref(ni), C.byref(mat))
            tan, bit = _FPtr(), _FPtr()
            self.lib.bm_model_mesh_tangents(self.h, i, C.byref(tan), C.byref(bit))
            v = nv.value

            def arr(ptr, k):
                return np.ctypeslib.as_array(ptr, shape=(v * k,)).reshape(v, k).copy() if ptr and v else None

            out.append({"pos": arr(pos, 3) if v else np.zeros((0, 3), np.float32), "nrm": arr(nrm, 3),
                        "uv": arr(uv, 2), "tan": arr(tan, 3), "bit": arr(bit, 3),
                        "idx": np.ctypeslib.as_array(idx, shape=(ni.value,)).copy() if ni.value else
                        np.zeros(0, np.uint32), "material": (mat.value or b"").decode()})
        return out

    def upload(self, ctx: "Context", scene: "IScene" = None, num_adds: int = 1):
        self.ctx = ctx
        ctx._check(self.lib.bm_model_upload(self.h, ctx.h, scene.h if scene is not None else None, num_adds))

    def gpu_mesh(self, i: int):
        return self.lib.bm_model_gpu_mesh(self.h, i)

    def destroy(self):
        if getattr(self, "h", None):
            self.lib.bm_model_destroy(self.h)
        self.h = None


_FPtr = C.POINTER(C.c_float)


def reachable_records(records: np.ndarray) -> np.ndarray:
    """Indices of the node records a traversal can reach from record 0 (BVH2, BVH4 or BVH8 layout)."""
    words = records.shape[1]
    ref_lo, nref = {64: (48, 8), 32: (24, 4)}.get(words, (12, 2))
    seen, stack = [], [0]
    mark = np.zeros(records.shape[0], bool)
    while stack:
        i = stack.pop()
        if mark[i]:
            continue
        mark[i] = True
        seen.append(i)
        for r in records[i, ref_lo:ref_lo + nref]:
            r = int(r)
            if r != 0xFFFFFFFF and not (r & 0x80000000):
                stack.append(r)
    return np.array(sorted(seen), np.int64)


def upload_meshes(ctx: Context, scene: IScene, meshes):
    """Create one IMesh per mesh dict {pos, nrm, idx} (Model::load order) and add it to scene."""
    out = []
    for m in meshes:
        mesh = IMesh.create(ctx)
        pos = _f32(m["pos"]).reshape(-1, 3)
        idx = np.ascontiguousarray(m["idx"], np.uint32).reshape(-1)
        ctx._check(mesh.setIndices(idx, idx.size))
        ctx._check(mesh.setVertexData(pos, pos.shape[0], 3, VERTEX_DATA_POSITION))
        if m.get("nrm") is not None:
            nrm = _f32(m["nrm"]).reshape(-1, 3)
            ctx._check(mesh.setVertexData(nrm, nrm.shape[0], 3, VERTEX_DATA_NORMAL))
        scene.addMesh(mesh)
        out.append(mesh)
    return out


def render(ctx: Context, meshes, width, height, rays, eye, orient, leaf_size=None):
    """Convenience: upload, build, trace one frame; returns (frame dict, build stats)."""
    scene = IScene.create(ctx)
    upload_meshes(ctx, scene, meshes)
    stats = scene.updateGPUScene(stats=True)
    cam = ICamera.create(ctx)
    ctx._check(cam.setInitialRays(width, height, *rays))
    rt = IRenderTarget.createOffscreen(ctx, width, height)
    ctx._check(cam.trace(eye, orient, scene, rt))
    frame = rt.read(rgb=True)
    rt.destroy()
    cam.destroy()
    scene.destroy()
    return frame, stats
