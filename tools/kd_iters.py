#!/usr/bin/env python3
"""Analysis only: per-ray iterations of the reference-mode march under the current node records and
under records that hold their children's boxes (tools/micro/kd_iters.c over the oracle's kd-tree),
per 8x8 wave (the lane maximum), for a config's frame.  python tools/kd_iters.py c2 [filled ...]"""
import ctypes as C
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle.oracle import Oracle, OrcMeshes, _p  # noqa: E402
from raytracercuda_amd import scenes  # noqa: E402

SRC = os.path.join(ROOT, "tools", "micro", "kd_iters.c")
LIB = os.path.join(ROOT, "tools", "micro", "libkd_iters.so")
if not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(SRC):
    subprocess.check_call(["gcc", "-O2", "-shared", "-fPIC", "-ffp-contract=off", "-o", LIB, SRC, "-lm"])
lib = C.CDLL(LIB)
o = Oracle()
for name in sys.argv[1:] or ["c2"]:
    c = scenes.CONFIGS[name]
    W, H = c["width"], c["height"]
    om = OrcMeshes(scenes.scene(c["scene"]))
    kd = o.lib.orc_kd_build(om.arr, om.count, -30.0, 30.0)
    err, rays = o.camera_rays(W, H, *c["rays"])
    out = np.zeros((W * H, 4), np.uint32)
    eye = np.asarray(c["eye"], np.float32)
    orient = np.asarray(scenes.IDENTITY, np.float32).reshape(9)
    lib.exp_kd_iters(C.c_void_p(kd), _p(rays, C.c_float), W * H, _p(eye, C.c_float), _p(orient, C.c_float),
                     _p(out, C.c_uint32))
    o.lib.orc_kd_free(C.c_void_p(kd))
    f = out.reshape(H, W, 4).astype(np.int64)
    th, tw = (H + 7) // 8, (W + 7) // 8
    pad = np.zeros((th * 8, tw * 8, 4), np.int64)
    pad[:H, :W] = f
    wmax = pad.reshape(th, 8, tw, 8, 4).max(axis=(1, 3)).reshape(-1, 4)
    print(f"{name}: per ray old {f[..., 0].mean():.2f} new {f[..., 1].mean():.2f} iterations, leaves {f[..., 2].mean():.2f}, "
          f"stack max {f[..., 3].max()}, p99.9 {np.percentile(f[..., 3], 99.9):.0f}")
    top = np.argsort(wmax[:, 0])[::-1][:10]
    print("  heaviest waves (lane-max old, new, leaves):", [tuple(int(v) for v in wmax[i, :3]) for i in top])
    print(f"  waves: lane-max old mean {wmax[:, 0].mean():.1f} max {wmax[:, 0].max()}, new mean {wmax[:, 1].mean():.1f} "
          f"max {wmax[:, 1].max()}")
