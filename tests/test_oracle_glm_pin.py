"""The oracle's scalar primitives pinned against the reference's own math library.

tests/golden/glm_pin.npz holds inputs and the values the reference's vendored glm 0.9.9.0
computes for them (oracle/glm_pin.cpp, tests/golden/make_glm_pin.py): orient * ray
(BuildTree.cu:377-378), 1/dir (:379), bmTriIntersect (CudaComon.cuh:117-155) and
bmFaceInterpolate<vec3> + normalize + pack (CudaComon.cuh:253-266, BuildTree.cu:489-491).
The oracle's C restatement (orc_pin_ops) must reproduce every output bit; the GPU kernels are
in turn bit-exact to the oracle on every frame (tests/test_gpu_*.py).
"""
import ctypes as C
import os
import subprocess
import tempfile

import numpy as np
import pytest

from oracle import Oracle

HERE = os.path.dirname(os.path.abspath(__file__))
FIX = os.path.join(HERE, "golden", "glm_pin.npz")
REPO = os.path.dirname(HERE)
GLM_BIN = os.path.join(REPO, "oracle", "_ref", "glm_pin")
FLT_MAX = np.float32(3.4028235e38)


def oracle_ops(inp):
    lib = Oracle().lib
    fn = lib.orc_pin_ops
    fn.argtypes = [C.c_uint32, C.POINTER(C.c_float), C.POINTER(C.c_float)]
    fn.restype = None
    inp = np.ascontiguousarray(inp, np.float32)
    out = np.zeros((inp.shape[0], 12), np.float32)
    fn(inp.shape[0], inp.ctypes.data_as(C.POINTER(C.c_float)), out.ctypes.data_as(C.POINTER(C.c_float)))
    return out


def same_bits(a, b):
    """Bit equality, NaN payloads included (both sides run the same IEEE operations)."""
    return np.array_equal(a.view(np.uint32), b.view(np.uint32))


def test_fixture_covers_hits_rejects_and_edge_cases():
    d = np.load(FIX)
    g = d["glm"]
    t = g[:, 6]
    assert (t != FLT_MAX).sum() > 1000 and (t == FLT_MAX).sum() > 500
    assert np.isinf(g[:, 3:6]).any(), "1/dir of zero components"
    assert np.isnan(g[:, 10]).any(), "normalize of a zero normal"


@pytest.mark.parametrize("what,cols", [("orient*ray", slice(0, 3)), ("1/dir", slice(3, 6)),
                                       ("bmTriIntersect t,u,v", slice(6, 9)), ("packed colour", slice(9, 10)),
                                       ("normalize(n).z", slice(10, 11))])
def test_oracle_primitives_equal_glm(what, cols):
    d = np.load(FIX)
    got = oracle_ops(d["inputs"])
    exp = d["glm"]
    bad = np.nonzero(~np.all(got[:, cols].view(np.uint32) == exp[:, cols].view(np.uint32), axis=1))[0]
    assert bad.size == 0, f"{what}: {bad.size} records differ from glm, first {bad[:5]}"


@pytest.mark.skipif(not os.path.isdir("/root/reference/3rdParty/glm-0.9.9.0"),
                    reason="the reference's glm is present only in the build container")
def test_fixture_is_what_glm_computes():
    """Rebuilds oracle/_ref/glm_pin from the reference's glm and re-derives the fixture's outputs."""
    subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle"), "glm_pin"], check=True)
    d = np.load(FIX)
    with tempfile.TemporaryDirectory() as td:
        a, b = os.path.join(td, "in.f32"), os.path.join(td, "out.f32")
        d["inputs"].tofile(a)
        subprocess.run([GLM_BIN, a, b], check=True)
        out = np.fromfile(b, np.float32).reshape(-1, 12)
    assert same_bits(out, d["glm"])
