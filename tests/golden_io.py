"""Helpers to read tests/golden fixtures (shared by CPU and GPU tests)."""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def manifest():
    return json.load(open(os.path.join(GOLDEN, "manifest.json")))


def view(name):
    with np.load(os.path.join(GOLDEN, "views", name + ".npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def sweep():
    with np.load(os.path.join(GOLDEN, "views", "bunny_sweep.npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def dense(n, rec, prefix="hit"):
    """Expand a sparse reference frame (hits only) to dense (packed, tri, t) arrays of n pixels."""
    packed = np.full(n, 0x0000FF00, np.uint32)
    tri = np.full(n, 0xFFFFFFFF, np.uint32)
    t = np.full(n, np.inf, np.float32)
    px = rec[f"{prefix}_pixels"]
    packed[px] = rec[f"{prefix}_packed"]
    tri[px] = rec[f"{prefix}_tri"]
    t[px] = rec[f"{prefix}_t"]
    return packed, tri, t


def closest_hit_expected(n, rec):
    """Reference frame with the early-out divergent pixels replaced by the closest-hit answer."""
    packed, tri, t = dense(n, rec)
    px = rec["div_pixels"]
    packed[px] = rec["div_packed"]
    tri[px] = rec["div_tri"]
    t[px] = rec["div_t"]
    return packed, tri, t
