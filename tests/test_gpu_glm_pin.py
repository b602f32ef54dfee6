"""The GPU's scalar primitives pinned against the reference's vendored glm 0.9.9.0.

bm_debug_primitives runs the device functions the trace kernels use — orient_mul (dir = orient *
ray, BuildTree.cu:377-378), 1/dir (:379), tri_test (bmTriIntersect, CudaComon.cuh:117-155, with the
trace's exact-safe reciprocal pre-reject) and shade_normals (bmFaceInterpolate<vec3> + normalize +
pack, CudaComon.cuh:253-266, BuildTree.cu:489-491) — on the records of tests/golden/glm_pin.npz,
whose expected values glm itself computed (oracle/glm_pin.cpp, tests/golden/make_glm_pin.py). Every
output bit must match, NaN payloads included; the degenerate, collinear, zero-direction and 1e+-30
records are where a pre-reject or a fused operation would show.
"""
import os

import numpy as np
import pytest

from raytracercuda_amd import beam

pytestmark = pytest.mark.gpu

FIX = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "glm_pin.npz")
COLS = [("orient*ray", slice(0, 3)), ("1/dir", slice(3, 6)), ("bmTriIntersect t,u,v", slice(6, 9)),
        ("packed colour", slice(9, 10)), ("normalize(n).z", slice(10, 11))]


@pytest.fixture(scope="module")
def gpu_out():
    d = np.load(FIX)
    ctx = beam.Context(device=0)
    out = ctx.debug_primitives(d["inputs"])
    ctx.close()
    return out, d["glm"]


@pytest.mark.parametrize("what,cols", COLS, ids=[c[0] for c in COLS])
def test_gpu_primitives_equal_glm(gpu_out, what, cols):
    got, exp = gpu_out
    bad = np.nonzero(~np.all(got[:, cols].view(np.uint32) == exp[:, cols].view(np.uint32), axis=1))[0]
    assert bad.size == 0, f"{what}: {bad.size} of {got.shape[0]} records differ from glm, first {bad[:5]}"


def test_gpu_primitives_empty_and_errors():
    ctx = beam.Context(device=0)
    assert ctx.debug_primitives(np.zeros((0, 36), np.float32)).shape == (0, 12)
    with pytest.raises(beam.BeamError):
        ctx._check(ctx.lib.bm_debug_primitives(ctx.h, 4, None, None))
    ctx.close()
