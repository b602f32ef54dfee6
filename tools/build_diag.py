#!/usr/bin/env python3
"""Active span of each LBVH build kernel (earliest workgroup start to latest wave end, s_memrealtime)
against the build's event time, from a diagnostic library (-DBM_BUILD_DIAG):

    python tools/build_ab.py raytracercuda_amd/libbeam_hip_bdiag.so BM_BUILD_DIAG=1   (CPU side)
    BEAM_HIP_LIB=$PWD/raytracercuda_amd/libbeam_hip_bdiag.so python tools/build_diag.py bunny,merged_proxy

The gap columns show where a build's time goes between kernels (dispatch, cache maintenance).
BDIAG_KD=1: the reference-mode kd build instead (its kernels' rows 9..15; the scans and the sort's
histogram kernel are not timed, so their time shows in the gaps)."""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools import ab_env  # noqa: E402
from raytracercuda_amd import _lib, beam, scenes  # noqa: E402

KD = os.environ.get("BDIAG_KD") == "1"
if KD:  # (row, kernel): rows 0..8 are bm_build.hip's (the sort's fourth pass lands in row 5), 9..15 bm_kd.hip's
    ROWS = [(0, "k_gather"), (9, "k_kd_top"), (10, "k_kd_sub count"), (12, "k_kd_copy"), (11, "k_kd_sub emit"),
            (2, "k_onesweep#0"), (3, "k_onesweep#1"), (4, "k_onesweep#2"), (5, "k_onesweep#3 (plain four-pass sort)"),
            (13, "k_kd_records")]
else:
    # small builds (n <= BM_MSD_MAX_N) run the top-digit pass (#2) first and k_bucket_sort in row 3
    ROWS = list(enumerate(["k_gather", "k_morton", "k_onesweep#0", "k_onesweep#1 | k_bucket_sort", "k_onesweep#2",
                           "k_span", "k_tree_chunk", "k_chunk_table", "k_pack4_span"]))
TICK_US = 0.01  # s_memrealtime: 100 MHz

lib = _lib.load()
fn = lib.bm_debug_build_diag
fn.argtypes = [C.c_void_p]
fn.restype = C.c_int32
KS, WS = 16, 1 << 16
WARM = os.environ.get("BDIAG_WARM") == "1"  # a ~0.2 ms busy kernel on the build's stream right before it
import torch  # noqa: E402
stream = torch.cuda.current_stream()
ctx = ab_env.Context(device=0, stream=stream.cuda_stream, reference_kd=KD)
a = torch.randn(2048, 2048, device="cuda")
for name in (sys.argv[1].split(",") if len(sys.argv) > 1 else ["bunny", "merged_proxy"]):
    sc = beam.IScene.create(ctx)
    keep = beam.upload_meshes(ctx, sc, scenes.scene(name))
    per, ms = [], []
    buf = np.zeros(KS * WS * 8, dtype=np.uint64)
    for it in range(10):
        assert fn(None) == 0
        if WARM:
            b = a @ a
        ms.append(sc.updateGPUScene(stats=True)["build_ms"])
        assert fn(buf.ctypes.data) == 0
        if it < 2:
            continue
        w = buf.reshape(KS, WS, 8).astype(np.float64)
        t0 = min(w[k, :, 0][w[k, :, 0] > 0].min() for k, _ in ROWS if (w[k, :, 0] > 0).any())
        row = []
        for k, _ in ROWS:
            st, en = w[k, :, 0], w[k, :, 1]
            ok = st > 0
            if not ok.any():
                row.append([np.nan] * 10)
                continue
            clk = (w[k, ok, 3] - w[k, ok, 2]) / np.maximum(w[k, ok, 1] - w[k, ok, 0], 1) * 100.0  # MHz
            st, en = (st[ok] - t0) * TICK_US, (en[ok] - t0) * TICK_US
            marks = []
            for mi in range(4):  # checkpoint i: median over waves of (mark - wave start), us
                mk = w[k, ok, 4 + mi]
                sel = mk > 0
                marks.append(float(np.median((mk[sel] - w[k, ok, 0][sel]) * TICK_US)) if sel.any() else np.nan)
            row.append([st.min(), en.max(), np.median(en - st), np.percentile(en, 50), float(ok.sum()),
                        np.median(clk)] + marks)
        per.append(row)
    r = np.nanmedian(np.array(per), axis=0)
    print(f"== front {sc.last_stats.get('fused_front')} {name}{' (warm)' if WARM else ''}: {sc.last_stats['num_tris']} tris, build_ms median "
          f"{np.median(ms[2:]) * 1e3:.1f} us (diagnostic build), first wave start -> last wave end "
          f"{np.nanmax(r[:, 1]):.1f} us", flush=True)
    prev = None
    order = sorted(range(len(ROWS)), key=lambda k: (np.isnan(r[k][0]), r[k][0]))  # in start order
    for k in order:
        nm = ROWS[k][1]
        s0, e0, wmed, emed, nw, clk = r[k][:6]
        mk = "  marks " + " ".join(f"{x:5.1f}" for x in r[k][6:] if not np.isnan(x)) if not np.all(np.isnan(r[k][6:])) else ""
        if np.isnan(s0):
            print(f"   {nm:16s} (not run)")
            continue
        gap = "" if prev is None else f"gap {s0 - prev:6.1f}"
        print(f"   {nm:16s} waves {int(nw):6d}  start {s0:7.1f}  half done {emed:7.1f}  end {e0:7.1f}  span "
              f"{e0 - s0:6.1f} us  wave median {wmed:6.1f} us  s_memtime rate {clk:7.1f} MHz  {gap}{mk}")
        prev = e0
    sc.destroy()
    del keep
ctx.close()
