"""C-ABI library: loads without a GPU, exports exactly what include/beam_c.h declares (CPU)."""
import ctypes as C
import os
import subprocess

import pytest

from raytracercuda_amd import _lib

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_header_declares_the_abi():
    names = _lib.declared_symbols()
    assert "bm_context_create" in names and "bm_camera_trace" in names
    assert set(names) == set(_lib.SIGNATURES), set(names) ^ set(_lib.SIGNATURES)


def test_library_exports_every_declared_symbol():
    lib = _lib.load()
    for name in _lib.declared_symbols():
        assert hasattr(lib, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = {ln.split()[-1] for ln in out.splitlines() if " T " in ln and ln.split()[-1].startswith("bm_")}
    assert exported == set(_lib.declared_symbols())


def test_version_and_null_handling_without_gpu_calls():
    lib = _lib.load()
    assert b"gfx950" in lib.bm_version()
    # every entry point rejects null handles before touching the device
    assert lib.bm_sync(None) == _lib.ERROR_INVALID_PARAMETER
    assert lib.bm_mesh_create(None, None) == _lib.ERROR_INVALID_PARAMETER
    assert lib.bm_scene_build(None, None) == _lib.ERROR_INVALID_PARAMETER
    assert lib.bm_camera_trace(None, None, None, None, None) == _lib.ERROR_INVALID_PARAMETER
    assert lib.bm_rt_read(None, None, None, None, None) == _lib.ERROR_INVALID_PARAMETER
    assert lib.bm_rt_lock(None) == _lib.ERROR_INVALID_PARAMETER
    assert lib.bm_context_create(None, None) == _lib.ERROR_INVALID_PARAMETER
    lib.bm_context_destroy(None)
    lib.bm_scene_destroy(None)


def test_cpp_header_compiles_against_the_abi(tmp_path):
    """include/beam/Beam.h (the reference-shaped C++ layer) compiles and links against the ABI."""
    src = os.path.join(REPO, "examples", "render_offscreen.cpp")
    if not os.path.exists(src):
        pytest.skip("example not present")
    exe = tmp_path / "render_offscreen"
    subprocess.run(["g++", "-std=c++17", "-O1", "-I", os.path.join(REPO, "include"), src, "-o", str(exe),
                    _lib.LIB_PATH, f"-Wl,-rpath,{os.path.dirname(_lib.LIB_PATH)}"], check=True)
    assert exe.exists()
