"""Per-wave statistics of the wave-packet trace (TRACE_PACKET, diagnostic build of k_trace_packet through
bm_camera_trace_profile): node and leaf steps per packet, lanes active per node step, triangle tests,
wave durations and the kernel's span; beside them the quad traversal's per-ray counters of the same
frame (the oracle's order).
    python tools/packet_stats.py c2 c3 filled c4"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from raytracercuda_amd import beam, scenes  # noqa: E402


def stats(cfg):
    c = scenes.CONFIGS[cfg]
    ctx = beam.Context(device=0, params={"trace_variant": 14})
    sc = beam.IScene.create(ctx)
    keep = beam.upload_meshes(ctx, sc, scenes.scene(c["scene"]))
    sc.updateGPUScene()
    cam = beam.ICamera.create(ctx)
    assert cam.setInitialRays(c["width"], c["height"], *c["rays"]) == 0
    rt = beam.IRenderTarget.createOffscreen(ctx, c["width"], c["height"])
    cnt = cam.traceCounters(c["eye"], scenes.IDENTITY, sc, rt)
    for _ in range(3):
        cam.trace(c["eye"], scenes.IDENTITY, sc, rt)
    d = cam.traceProfile(c["eye"], scenes.IDENTITY, sc, rt).astype(np.int64)
    t0, t1 = d[:, 0], d[:, 1]
    nodes, leaves = d[:, 2] & 0xFFFFFFFF, d[:, 2] >> 32
    lanes, tris = d[:, 3] & 0xFFFFFFFF, d[:, 3] >> 32
    dur = (t1 - t0) * 10 / 1000  # 100 MHz ticks -> us
    span = (t1.max() - t0.min()) * 10 / 1000
    busy = nodes > 1
    rays = c["width"] * c["height"]
    q = lambda a, p: float(np.percentile(a, p)) if a.size else 0.0  # noqa: E731
    print(f"{cfg}: {len(d)} packets, span {span:.1f} us; {busy.sum()} with more than the root "
          f"({busy.mean():.1%}); quad order per ray: {cnt[0] / rays:.2f} node records, {cnt[1] / rays:.2f} tri tests")
    nb, lb, tb, lab, db = nodes[busy], leaves[busy], tris[busy], lanes[busy], dur[busy]
    print(f"   per busy packet: node steps mean {nb.mean():.1f} p50 {q(nb, 50):.0f} p90 {q(nb, 90):.0f} max {nb.max()}; "
          f"leaf steps mean {lb.mean():.1f} max {lb.max()}; tri tests mean {tb.mean():.1f}")
    print(f"   active lanes per node step {lab.sum() / max(nb.sum(), 1):.1f} of 64; "
          f"wave us mean {db.mean():.2f} p50 {q(db, 50):.2f} p90 {q(db, 90):.2f} max {db.max():.2f}; "
          f"us per step {db.sum() / max((nb + lb).sum(), 1):.3f}")
    print(f"   total wave steps {int((nodes + leaves).sum())} (nodes {int(nodes.sum())}, leaves {int(leaves.sum())}); "
          f"quad wave steps (per-ray records / 16) ~{int((cnt[0] + cnt[1] / 4) / 16)}")
    rt.destroy()
    cam.destroy()
    sc.destroy()
    del keep
    ctx.close()


if __name__ == "__main__":
    for cfg in sys.argv[1:] or ["c2", "c3", "filled", "c4"]:
        stats(cfg)
