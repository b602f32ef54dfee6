#!/usr/bin/env python3
"""Generate tests/golden/glm_pin.npz: inputs for the scalar primitives of the hot path and their
values computed by the reference's vendored glm 0.9.9.0 (oracle/glm_pin.cpp, built by
`make -C oracle glm_pin` from /root/reference/3rdParty/glm-0.9.9.0 unmodified).

Run in this container only (it needs /root/reference); the test reads the committed npz.

    python tests/golden/make_glm_pin.py

Records (oracle/beam_oracle.c orc_pin_ops): a ray from `orig` along orient*ray at a triangle,
normals to interpolate at (su, sv). Rays are aimed at a point of the triangle (about half hit, the
rest fall just outside an edge), plus edge cases: zero and negative-zero direction components
(1/dir = +-inf), degenerate triangles (det = 0), rays from a vertex, tiny and large coordinates,
(su, sv) on the edges of the barycentric range and zero normals (normalize of 0: NaN).
"""
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
BIN = os.path.join(REPO, "oracle", "_ref", "glm_pin")


def records(n_rand=3072, seed=20261016):
    rng = np.random.default_rng(seed)
    f = np.float32
    recs = []
    for i in range(n_rand):
        scale = f(10.0 ** rng.uniform(-3, 2))
        v = (rng.uniform(-1, 1, (3, 3)) * scale).astype(f)
        orig = (rng.uniform(-3, 3, 3) * scale).astype(f)
        q, _ = np.linalg.qr(rng.normal(size=(3, 3)))
        m = (q * rng.choice([1, -1], 3)).astype(f)  # m[:, c] = column c
        b = rng.dirichlet([1, 1, 1]) * (1.0 + rng.uniform(-0.3, 0.3))  # some outside the triangle
        target = (b[0] * v[0] + b[1] * v[1] + b[2] * v[2]).astype(np.float64)
        dw = target - orig
        ray = (m.astype(np.float64).T @ dw)
        ray = (ray / np.linalg.norm(ray)).astype(f)
        nrm = rng.normal(size=(3, 3)).astype(f)
        su, sv = rng.uniform(0, 1, 2).astype(f)
        recs.append(np.concatenate([orig, ray, m.T.reshape(-1), v.reshape(-1), nrm.reshape(-1), [su, sv, 0]]))
    base = recs[0].copy()
    edge = []
    for comp in range(3):  # zero / negative-zero ray components through the identity orient
        for z in (0.0, -0.0):
            r = base.copy()
            r[6:15] = np.eye(3, dtype=f).reshape(-1)
            r[3:6] = [0.3, -0.4, 0.5]
            r[3 + comp] = z
            edge.append(r)
    r = base.copy()
    r[18:21] = r[15:18]  # degenerate: v1 == v0
    edge.append(r)
    r = base.copy()
    r[21:24] = r[15:18] + 2 * (r[18:21] - r[15:18])  # collinear vertices
    edge.append(r)
    r = base.copy()
    r[0:3] = r[15:18]  # ray from a vertex
    edge.append(r)
    for su, sv in ((0, 0), (1, 0), (0, 1), (0.5, 0.5), (1e-8, 1 - 1e-8)):
        r = base.copy()
        r[33:35] = [su, sv]
        edge.append(r)
    r = base.copy()
    r[24:33] = 0  # zero normals
    edge.append(r)
    r = base.copy()
    r[15:24] *= f(1e-30)
    r[0:3] *= f(1e-30)
    edge.append(r)
    r = base.copy()
    r[15:24] *= f(1e30)
    r[0:3] *= f(1e30)
    edge.append(r)
    return np.ascontiguousarray(np.stack(recs + edge).astype(np.float32))


def glm_outputs(inp):
    with tempfile.TemporaryDirectory() as d:
        a, b = os.path.join(d, "in.f32"), os.path.join(d, "out.f32")
        inp.tofile(a)
        subprocess.run([BIN, a, b], check=True)
        return np.fromfile(b, np.float32).reshape(-1, 12)


def main():
    if not os.path.exists(BIN):
        subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle"), "glm_pin"], check=True)
    inp = records()
    out = glm_outputs(inp)
    hits = int((out[:, 6] != np.float32(3.4028235e38)).sum())
    np.savez_compressed(os.path.join(HERE, "glm_pin.npz"), inputs=inp, glm=out)
    print(f"glm_pin.npz: {inp.shape[0]} records, {hits} triangle hits", file=sys.stderr)


if __name__ == "__main__":
    main()
