"""ctypes binding of libbeam_hip.so (the C ABI declared in include/beam_c.h).

The product path has no fallback: if the HIP library is missing or cannot load, importing the
binding raises, and a context on a machine without a usable GPU returns BM_ERROR_DEVICE.
"""
from __future__ import annotations

import ctypes as C
import os
import re

PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(PKG, "libbeam_hip.so")
HEADER = os.path.join(os.path.dirname(PKG), "include", "beam_c.h")

ERROR_ALL_FINE = 0
ERROR_NO_VERTICES = 1
ERROR_INVALID_PARAMETER = 2
ERROR_GPU_ALLOC_FAIL = 3
ERROR_INVALID_FORMAT = 4
ERROR_RT_CAM_MISMATCH = 5
ERROR_UNLOCK_FIRST = 6
ERROR_LOCK_FIRST = 7
ERROR_NO_RENDER_TARGET = 8
ERROR_DEVICE = 9
ERROR_NOT_BUILT = 10

VERTEX_DATA_POSITION = 0
VERTEX_DATA_NORMAL = 1
VERTEX_DATA_COUNT = 10
OPT_NULL_STREAM = 1
OPT_SHADOW_QUEUE = 2
OPT_BVH2 = 4
OBJ_UNSHARED = 1
OPT_REFERENCE_KD = 8
OPT_REFERENCE_HASH = 16
OPT_BVH8 = 32
MISS_PACKED = 0x0000FF00
NO_TRIANGLE = 0xFFFFFFFF


class BeamError(RuntimeError):
    def __init__(self, code, msg=""):
        super().__init__(f"beam error {code}: {msg}")
        self.code = code


MAX_DEVICES = 8
COMM_ID_BYTES = 128
GATHER_AUTO, GATHER_PEER, GATHER_RCCL, GATHER_RCCL_LOOPBACK = 0, 1, 2, 3
PLANE_PACKED, PLANE_TRI_ID, PLANE_T, PLANE_NZ, PLANE_SHADOW = 1, 2, 4, 8, 16


class Options(C.Structure):
    _fields_ = [("device", C.c_int32), ("stream", C.c_void_p), ("leaf_size", C.c_uint32), ("flags", C.c_uint32),
                ("num_devices", C.c_uint32), ("devices", C.c_int32 * MAX_DEVICES), ("band_height", C.c_uint32),
                ("gather", C.c_uint32), ("gather_planes", C.c_uint32), ("comm_rank", C.c_int32),
                ("comm_size", C.c_int32), ("comm_id", C.c_uint8 * COMM_ID_BYTES)]


class ModelInfo(C.Structure):
    _fields_ = [("num_meshes", C.c_uint32), ("num_faces", C.c_uint64), ("num_vertices", C.c_uint64),
                ("bmin", C.c_float * 3), ("bmax", C.c_float * 3)]


class BuildStats(C.Structure):
    _fields_ = [("num_meshes", C.c_uint32), ("num_tris", C.c_uint32), ("num_records", C.c_uint32),
                ("leaf_size", C.c_uint32), ("build_ms", C.c_float), ("bvh_width", C.c_uint32),
                ("sort_path", C.c_uint32), ("fused_front", C.c_uint32)]


SORT_LSD, SORT_MSD, SORT_MSD_SKEW, SORT_KD_RANKED = 1, 2, 3, 4

# bm_context_set_param keys (BM_PARAM_* in include/beam_c.h), by the names beam.Context(params=...) takes
PARAMS = {"trace_variant": 0, "trace_sched": 1, "trace_scramble": 2, "trace_prio_after": 3, "trace_prio_level": 4,
          "trace_refill_min": 5, "cull_tiles": 6, "trace_auto_compact": 7, "trace_grid": 8, "readback_sync": 9,
          "kd_queue_cap": 10, "kd_lq_cap": 11, "kd_split": 12, "kd_grid": 13, "kd_pair": 14, "kd_tb": 15,
          "kd_march": 16, "msd_max_n": 17, "nrm_defer": 18, "bucket_lds_cap": 19, "msd_wide_n": 20,
          "front_max_n": 21, "orig_lazy": 22, "kd_max_leaves": 23,
          "trace_auto_packet": 24, "kd_top_rank": 25}


_P = C.c_void_p
_I = C.c_int32
_U = C.c_uint32
_F = C.c_float
_FP = C.POINTER(C.c_float)
_UP = C.POINTER(C.c_uint32)
_U64P = C.POINTER(C.c_uint64)

# name: (restype, argtypes) — every function declared in include/beam_c.h
SIGNATURES = {
    "bm_context_create": (_I, [C.POINTER(Options), C.POINTER(_P)]),
    "bm_context_destroy": (None, [_P]),
    "bm_sync": (_I, [_P]),
    "bm_last_error_string": (C.c_char_p, [_P]),
    "bm_context_stream": (_P, [_P]),
    "bm_version": (C.c_char_p, []),
    "bm_context_num_devices": (_U, [_P]),
    "bm_comm_unique_id": (_I, [C.POINTER(C.c_uint8)]),
    "bm_comm_available": (_I, []),
    "bm_context_gather": (_U, [_P]),
    "bm_context_start_comm": (_I, [_P, _I, _I, C.POINTER(C.c_uint8)]),
    "bm_context_set_param": (_I, [_P, _U, C.c_int64]),
    "bm_context_get_param": (C.c_int64, [_P, _U]),
    "bm_rt_last_timing": (_I, [_P, _FP]),
    "bm_mesh_create": (_I, [_P, C.POINTER(_P)]),
    "bm_mesh_set_vertex_data": (_I, [_P, _FP, _U, _U, _U]),
    "bm_mesh_set_indices": (_I, [_P, _UP, _U]),
    "bm_mesh_destroy": (None, [_P]),
    "bm_scene_create": (_I, [_P, C.POINTER(_P)]),
    "bm_scene_add_mesh": (_I, [_P, _P]),
    "bm_scene_remove_mesh": (_I, [_P, _P]),
    "bm_scene_build": (_I, [_P, C.POINTER(BuildStats)]),
    "bm_scene_refit": (_I, [_P, C.POINTER(BuildStats)]),
    "bm_scene_kd_stats": (_I, [_P, _U64P]),
    "bm_scene_grid_stats": (_I, [_P, _U64P]),
    "bm_scene_grid_export": (_I, [_P, _UP, _UP, _UP]),
    "bm_model_load": (_I, [C.c_char_p, _U, C.POINTER(_P)]),
    "bm_model_info_get": (_I, [_P, C.POINTER(ModelInfo)]),
    "bm_model_mesh": (_I, [_P, _U, C.POINTER(_FP), C.POINTER(_FP), C.POINTER(_FP), C.POINTER(_UP), C.POINTER(_U),
                           C.POINTER(_U), C.POINTER(C.c_char_p)]),
    "bm_model_mesh_tangents": (_I, [_P, _U, C.POINTER(_FP), C.POINTER(_FP)]),
    "bm_model_upload": (_I, [_P, _P, _P, _U]),
    "bm_model_gpu_mesh": (_P, [_P, _U]),
    "bm_model_destroy": (None, [_P]),
    "bm_scene_destroy": (None, [_P]),
    "bm_camera_create": (_I, [_P, C.POINTER(_P)]),
    "bm_camera_set_initial_rays": (_I, [_P, _U, _U, _F, _F, _F, _F, _F]),
    "bm_camera_trace": (_I, [_P, _FP, _FP, _P, _P]),
    "bm_camera_trace_bands": (_I, [_P, _FP, _FP, _P, _P, _U, _U, _U]),
    "bm_camera_trace_shadow": (_I, [_P, _FP, _FP, _P, _P, _FP]),
    "bm_camera_trace_shadow_bands": (_I, [_P, _FP, _FP, _P, _P, _U, _U, _U, _FP]),
    "bm_camera_destroy": (None, [_P]),
    "bm_rt_create_offscreen": (_I, [_P, _U, _U, _U, C.POINTER(_P)]),
    "bm_rt_create_external": (_I, [_P, _U, _U, _U, _P, _P, _P, _P, C.POINTER(_P)]),
    "bm_rt_width": (_U, [_P]),
    "bm_rt_height": (_U, [_P]),
    "bm_rt_pitch": (_U, [_P]),
    "bm_rt_buffer": (_P, [_P]),
    "bm_rt_tri_id": (_P, [_P]),
    "bm_rt_t": (_P, [_P]),
    "bm_rt_nz": (_P, [_P]),
    "bm_rt_shadow": (_P, [_P]),
    "bm_rt_lock": (_I, [_P]),
    "bm_rt_unlock": (_I, [_P]),
    "bm_rt_clear": (_I, [_P, _U]),
    "bm_rt_read": (_I, [_P, _UP, _UP, _FP, _FP]),
    "bm_rt_save_ppm": (_I, [_P, C.c_char_p]),
    "bm_debug_primitives": (_I, [_P, C.c_uint32, C.c_void_p, C.c_void_p]),
    "bm_rt_set_stream": (_I, [_P, _P]),
    "bm_rt_stream": (_P, [_P]),
    "bm_rt_trace_kind": (_I, [_P]),
    "bm_rt_read_shadow": (_I, [_P, C.POINTER(C.c_uint8)]),
    "bm_rt_destroy": (None, [_P]),
    "bm_camera_trace_counters": (_I, [_P, _FP, _FP, _P, _P, _U64P]),
    "bm_camera_trace_shadow_counters": (_I, [_P, _FP, _FP, _P, _P, _FP, _U64P]),
    "bm_scene_export": (_I, [_P, _UP, _UP, _UP, _UP]),
    "bm_camera_trace_profile": (_I, [_P, _FP, _FP, _P, _P, _U64P, _U, _UP]),
}


def declared_symbols(header: str = HEADER):
    """Function names declared in include/beam_c.h."""
    text = open(header).read()
    return sorted(set(re.findall(r"^\s*(?:[\w\*\s]+?)\b(bm_\w+)\s*\(", text, re.M)))


_lib = None


def load(path: str = LIB_PATH) -> C.CDLL:
    """Load the HIP library (building it first if the sources are newer). Raises if unavailable.
    BEAM_HIP_LIB names another build of the same library (A/B timing of an older build only)."""
    global _lib
    if _lib is not None:
        return _lib
    ab = os.environ.get("BEAM_HIP_LIB")
    if ab:
        lib = C.CDLL(ab, mode=C.RTLD_GLOBAL)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name, None)
            if fn is not None:
                fn.restype = res
                fn.argtypes = args
        _lib = lib
        return _lib
    if not os.path.exists(path) or path == LIB_PATH:
        try:
            from . import build as _build  # compile in-tree when hipcc is present and the build is stale
            _build.build()
        except Exception as e:  # noqa: BLE001
            if not os.path.exists(path):
                raise ImportError(f"libbeam_hip.so missing and could not be built: {e}") from e
            import sys
            print(f"warning: libbeam_hip.so does not match the sources and could not be rebuilt ({e}); "
                  f"loading the existing build", file=sys.stderr)
    lib = C.CDLL(path, mode=C.RTLD_GLOBAL)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib
