#!/usr/bin/env python3
"""Benchmark: Mrays/s of 1920x1080 primary rays (+ BVH build ms) on 1..8 MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--scene bunny] [--no-cpu-baseline]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

Workload (BASELINE.json configs[1]): the Stanford bunny of the reference's Content/bunny.zip
(69,630 triangles, committed as tests/golden/meshes/bunny.npz), camera eye (-0.34, 1.2, -3.5),
setInitialRays(1920, 1080, -16/9, 16/9, -1, 1, 1). A step = one primary-ray trace of the frame
with the BVH resident in HBM (inputs resident before the timed region). Frames in flight
(--frames-in-flight, default 3): consecutive steps trace into alternating render targets, each on
its own HIP stream (bm_rt_set_stream), so one frame's trace starts while the previous one drains;
`value` is the steady-state rate, `trace_kernel_ms` the kernel span measured per launch with HIP
events on its own stream (it includes the time a launch shares the CUs with its neighbour). At N GPUs the frame is
1920 x (1080*N) over the same field of view (N vertical samples per 1080p pixel), cut into 16-row
bands dealt round-robin to the ranks, each rank tracing 1920x1080 rays; a step then also includes
the single RCCL gather of every rank's band buffer (12 B/pixel) into rank 0 — weak scaling.

One JSON line on rank 0 (driver contract), with `roofline` (dominant kernel: the trace) and
`cpu_baseline` (the scalar CPU LBVH of oracle/, same algorithm and arithmetic, on up to 16 host
threads; the one-thread figure beside it).
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)
BAND_H = 16
TRACE_KERNEL = "k_trace_quad<false"  # the timed (non-counting) trace kernel (ray quads, the default variant)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--scene", default="bunny")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--leaf-size", type=int, default=4)
    ap.add_argument("--bvh-width", type=int, default=4, choices=(2, 4))
    ap.add_argument("--gather-planes", default="packed", choices=("packed", "full"),
                    help="multi-GPU: gather the framebuffer (4 B/px) or packed+id+t (12 B/px)")
    ap.add_argument("--frames-in-flight", type=int, default=3,
                    help="band buffers / render targets, each on its own HIP stream (1: every frame on one stream)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extra", action="store_true", help="skip the armadillo-proxy side measurement")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    return ap.parse_args()


def algorithmic_bytes(counters, rays, bvh_width=4):
    """SURVEY.md §8(d) per-ray bytes, with this layout: per node record fetched 64 B (BVH2) or
    112 B (BVH4: six 16-B SoA box planes + refs), 48 B per triangle record tested, 36 B of corner
    normals per hit, 8 B of camera tables per ray (rx, ry), 12 B of output per ray (packed,
    triangle id, t)."""
    nodes, tris, hits = (int(x) for x in counters)
    return (112 if bvh_width == 4 else 64) * nodes + 48 * tris + 36 * hits + (8 + 12) * rays


def cpu_threads():
    """Host threads for the CPU baseline: the cores this process may run on, capped at 16 (the GPU
    box's CPU share per GPU; os.cpu_count() there reports the whole machine)."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def cpu_baseline(meshes, width, height, cam, eye, orient, seconds, bvh_width=4):
    """Scalar CPU LBVH (oracle/, the same algorithm and arithmetic as the HIP path) on the host
    cores: full frames with the rows split into contiguous ranges over T threads (ctypes releases
    the GIL inside orc_bvh_trace), repeated until `seconds` of wall time; plus the same on one
    thread for ~seconds/3 (one thread and all host cores)."""
    from concurrent.futures import ThreadPoolExecutor

    from oracle import Oracle
    o = Oracle()
    err, rays = o.camera_rays(width, height, *cam)
    n = rays.shape[0]
    t0 = time.perf_counter()
    bvh = o.bvh_build(meshes, 4, bvh_width)
    build_s = time.perf_counter() - t0

    def run(threads, budget):
        done, el = 0, 0.0
        cuts = np.linspace(0, n, 8 * threads + 1).astype(np.int64)  # 8 chunks per thread
        with ThreadPoolExecutor(max_workers=threads) as pool:
            while el < budget:
                t0 = time.perf_counter()
                if threads == 1:
                    bvh.render(rays, eye, orient)
                else:
                    list(pool.map(lambda k: bvh.render(rays, eye, orient, int(cuts[k]), int(cuts[k + 1])),
                                  range(len(cuts) - 1)))
                el += time.perf_counter() - t0
                done += n
        return done, el

    d1, e1 = run(1, seconds / 3)
    T = cpu_threads()
    dT, eT = run(T, seconds) if T > 1 else (d1, e1)
    cpu = "unknown"
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                cpu = ln.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"value": dT / eT / 1e6, "unit": "Mrays/s", "cores": T, "kind": "port",
            "sample": f"{dT // n} full {width}x{height} frames ({dT} rays, {eT:.1f} s) on {T} threads "
                      f"(rows split 8 ranges/thread) + {d1 // n} frames on 1 thread ({e1:.1f} s); scalar oracle "
                      f"LBVH (BVH{bvh_width}) closest-hit trace; build {build_s * 1e3:.0f} ms (1 thread)",
            "single_thread_mrays_s": d1 / e1 / 1e6,
            "build_ms": build_s * 1e3, "cpu_model": cpu, "host_threads": os.cpu_count()}


def shadow_side_figure(ctx, cam, stream, W, H, eye, orient):
    """SURVEY §8(d) C5 on one GPU: tyra+f16 proxy (1,118,136 tris), 1080p primary rays + one any-hit
    shadow ray per hit toward (0,10,-10); frame time covers both passes."""
    import torch

    from raytracercuda_amd import beam, scenes
    light = (0.0, 10.0, -10.0)
    sm = beam.IScene.create(ctx)
    keep = beam.upload_meshes(ctx, sm, scenes.scene("merged_proxy"))
    builds = [sm.updateGPUScene(stats=True)["build_ms"] for _ in range(5)]
    rt = beam.IRenderTarget.createOffscreen(ctx, W, H)
    cnt = cam.traceShadowCounters(eye, orient, sm, rt, light)
    res = {}
    for name, fn in (("primary", lambda: cam.trace(eye, orient, sm, rt)),
                     ("primary+shadow", lambda: cam.traceShadow(eye, orient, sm, rt, light))):
        for _ in range(5):
            ctx._check(fn())
        torch.cuda.synchronize()
        ea, eb = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ea.record(stream)
        for _ in range(20):
            ctx._check(fn())
        eb.record(stream)
        torch.cuda.synchronize()
        res[name] = ea.elapsed_time(eb) / 20
    rt.destroy()
    sm.destroy()
    del keep
    hits, shadowed = int(cnt[2]), int(cnt[5])
    return {"tris": 1118136, "light": list(light), "build_ms": float(np.median(builds[1:])),
            "primary_ms": res["primary"], "frame_ms": res["primary+shadow"], "shadow_rays": hits,
            "shadowed": shadowed, "shadow_pass_ms": res["primary+shadow"] - res["primary"],
            "rays_per_s_M": (W * H + hits) / (res["primary+shadow"] / 1e3) / 1e6,
            "shadow_per_ray": {"node_records": float(cnt[3]) / max(hits, 1),
                               "tri_tests": float(cnt[4]) / max(hits, 1)}}


def reference_side_figure(device, stream, meshes, W, H, cam_rays, eye, orient, mode="kd"):
    """Reference mode on the bench frame: mode "kd" (BM_OPT_REFERENCE_KD) = the reference's kd-tree
    build and first-hit-leaf march on the GPU, every pixel equal to the reference framebuffer;
    mode "hash" (BM_OPT_REFERENCE_HASH) = its alternative hashed uniform grid (Hash.cu)."""
    import torch

    from raytracercuda_amd import beam
    ctx = beam.Context(device=device, stream=stream.cuda_stream, reference_kd=mode == "kd",
                       reference_hash=mode == "hash")
    sc = beam.IScene.create(ctx)
    keep = beam.upload_meshes(ctx, sc, meshes)
    builds = [sc.updateGPUScene(stats=True)["build_ms"] for _ in range(4)]
    cam = beam.ICamera.create(ctx)
    ctx._check(cam.setInitialRays(W, H, *cam_rays))
    rt = beam.IRenderTarget.createOffscreen(ctx, W, H)
    for _ in range(3):
        ctx._check(cam.trace(eye, orient, sc, rt))
    torch.cuda.synchronize()
    ea, eb = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ea.record(stream)
    for _ in range(10):
        ctx._check(cam.trace(eye, orient, sc, rt))
    eb.record(stream)
    torch.cuda.synchronize()
    ms = ea.elapsed_time(eb) / 10
    st = sc.kdStats() if mode == "kd" else sc.gridStats()
    hits = int((rt.read(tri_id=False, t=False)["packed"] != 0x0000FF00).sum())
    rt.destroy()
    cam.destroy()
    sc.destroy()
    del keep
    ctx.close()
    out = {"build_ms": float(np.median(builds[1:])), "trace_ms": ms, "mrays_s": W * H / (ms / 1e3) / 1e6,
           "frame_hits": hits}
    if mode == "kd":
        out.update({"kd_leaves": int(st[0]), "face_refs": int(st[1])})
    else:
        out.update({"cell_face_pairs": int(st[0]), "buckets_used": int(st[1]), "largest_bucket": int(st[2]),
                    "dropped_by_cap": int(st[3])})
    return out


def measured_traffic(kernel_prefix):
    """HBM bytes per launch of the timed kernel from the newest committed PMC summary
    (profiles/*_traffic.json, written by tools/summarize_profile.py from separate rocprofv3 --pmc
    FETCH_SIZE / WRITE_SIZE passes of this same command; FETCH_SIZE doubled per the gfx950 note)."""
    import glob
    import re
    # newest = highest round, then highest profile number (r01_v10 after r01_v9: numeric, not lexical)
    files = sorted(glob.glob(os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "*_traffic.json")),
                   key=lambda f: [int(x) for x in re.findall(r"\d+", os.path.basename(f))])
    if not files:
        return None, None
    d = json.load(open(files[-1]))
    for k, v in d.get("kernels", {}).items():
        if k.startswith(kernel_prefix) and v.get("read_bytes_x2") is not None and v.get("write_bytes") is not None:
            return float(v["read_bytes_x2"] + v["write_bytes"]), os.path.relpath(files[-1],
                                                                                 os.path.dirname(files[-1]) + "/..")
    return None, None


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    from raytracercuda_amd import beam, multigpu, scenes

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE", file=sys.stderr)
    # BM_BENCH_SHARED_DEVICE=1: rehearsal of the N-rank path on a 1-GPU box — every rank on
    # cuda:0, gloo instead of RCCL (the gather stages through host memory). Never used for results.
    shared = os.environ.get("BM_BENCH_SHARED_DEVICE") == "1"
    if shared:
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if shared:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)

    stream = torch.cuda.current_stream()
    ctx = beam.Context(device=local, stream=stream.cuda_stream, leaf_size=args.leaf_size, bvh_width=args.bvh_width)
    meshes = scenes.scene(args.scene)
    scene = beam.IScene.create(ctx)
    keep = beam.upload_meshes(ctx, scene, meshes)
    # BVH build: median device time over repeated rebuilds (first one allocates)
    build_ms = []
    for _ in range(7):
        build_ms.append(scene.updateGPUScene(stats=True)["build_ms"])
    st = scene.last_stats
    build_med = float(np.median(build_ms[2:]))

    W = args.width
    H = args.height * world
    cam_rays = scenes.RAYS_1080 if (args.width, args.height) == (1920, 1080) else (
        -args.width / args.height, args.width / args.height, -1.0, 1.0, 1.0)
    eye, orient = scenes.BUNNY_EYE, scenes.IDENTITY
    cam = beam.ICamera.create(ctx)
    ctx._check(cam.setInitialRays(W, H, *cam_rays))
    br = multigpu.BandRenderer(ctx, scene, cam, W, H, BAND_H, rank, world, dev, planes=args.gather_planes,
                               frames_in_flight=args.frames_in_flight)
    rays_per_rank = W * args.height

    # algorithmic-bytes counters (untimed, deterministic)
    rt_cnt = beam.IRenderTarget.createOffscreen(ctx, W, H)
    counters = cam.traceCounters(eye, orient, scene, rt_cnt)
    rt_cnt.destroy()
    frame_bytes = algorithmic_bytes(counters, W * H, st["bvh_width"])

    def step():
        ctx._check(br.trace(eye, orient))
        br.gather()

    for _ in range(args.warmup):
        step()
    # trace-kernel duration with events on the stream the kernel runs on (torch's current stream)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        br.acquire()  # outside the kernel-time events: waits (on the stream) for the gather 2 steps back
        fst = br.stream()  # the stream this frame's trace is enqueued on (its render target's)
        ev[i][0].record(fst)
        ctx._check(br.trace(eye, orient))
        ev[i][1].record(fst)
        br.gather()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    if world > 1:
        t = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device="cpu" if shared else dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_ms_max = float(t[0]), float(t[1])
    else:
        kern_ms_max = kern_ms

    # parity spot check of the benchmarked frame (rank 0): hit count vs the committed fixture
    extra = {}
    if rank == 0:
        fr = br.frame()
        hits = int((fr[0] != 0x0000FF00).sum().item())  # packed plane: miss colour is 0xFF00
        extra["frame_hits"] = hits
        if world > 1:
            # the assembled multi-GPU frame must equal this GPU's own full-frame trace, bit for bit
            rt_full = beam.IRenderTarget.createOffscreen(ctx, W, H)
            ctx._check(cam.trace(eye, orient, scene, rt_full))
            full = rt_full.read()
            rt_full.destroy()
            got = fr.cpu().numpy()
            ok = np.array_equal(got[0].view(np.uint32), full["packed"])
            if got.shape[0] == 3:
                ok = ok and np.array_equal(got[1].view(np.uint32), full["tri_id"]) and \
                    np.array_equal(got[2].view(np.float32), full["t"])
            extra["frame_check"] = bool(ok)
            extra["gather_planes"] = args.gather_planes

    total_rays = rays_per_rank * world * args.steps
    value = total_rays / elapsed / 1e6
    # roofline of the dominant kernel: bytes of one launch (this rank's share of the frame)
    bytes_launch = frame_bytes / world
    achieved = bytes_launch / (kern_ms / 1e3) / 1e9

    if rank == 0 and world == 1 and not args.no_extra:
        # side measurement: armadillo proxy (278,520 tris), north_star target config, 1 GPU
        am = scenes.scene("armadillo_proxy")
        sa = beam.IScene.create(ctx)
        ka = beam.upload_meshes(ctx, sa, am)
        abuild = [sa.updateGPUScene(stats=True)["build_ms"] for _ in range(5)]
        rta = beam.IRenderTarget.createOffscreen(ctx, W, H)
        for _ in range(5):
            ctx._check(cam.trace(eye, orient, sa, rta))
        torch.cuda.synchronize()
        ea, eb = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ea.record(stream)
        for _ in range(20):
            ctx._check(cam.trace(eye, orient, sa, rta))
        eb.record(stream)
        torch.cuda.synchronize()
        ams = ea.elapsed_time(eb) / 20
        extra["armadillo_proxy"] = {"tris": 278520, "mrays_s": W * H / (ams / 1e3) / 1e6,
                                    "trace_ms": ams, "build_ms": float(np.median(abuild[1:]))}
        rta.destroy()
        sa.destroy()
        extra["merged_proxy_shadow"] = shadow_side_figure(ctx, cam, stream, W, H, eye, orient)
        extra["reference_mode"] = reference_side_figure(local, stream, meshes, W, H, cam_rays, eye, orient)
        extra["hashed_grid"] = reference_side_figure(local, stream, meshes, W, H, cam_rays, eye, orient, "hash")

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(meshes, W, H, cam_rays, eye, orient, args.cpu_seconds, st["bvh_width"])

    traffic, traffic_src = measured_traffic(TRACE_KERNEL)
    if traffic is not None and world > 1:
        traffic = None  # the committed PMC pass is the 1-GPU frame
    if rank == 0:
        out = {
            "metric": "Mrays/s primary rays @1920x1080 + BVH build ms, 1/2/4/8 MI355X",
            "value": value,
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic pinhole camera rays over the reference's Stanford bunny mesh (Content/bunny.zip)",
            "config": {
                "workload": f"{args.scene} ({st['num_tris']} tris) {W}x{args.height} primary rays per GPU; "
                            f"frame {W}x{H}, {BAND_H}-row bands round-robin over {world} GPU(s)"
                            + (", RCCL gather to rank 0" if world > 1 else "")
                            + f"; {br.nbuf} frames in flight (one HIP stream per render target)",
                "scene": args.scene, "tris": st["num_tris"], "width": W, "height": H, "band_h": BAND_H,
                "leaf_size": st["leaf_size"], "bvh_width": st["bvh_width"],
                "parallelism": f"screen-bands x{world}",
            },
            "build_ms": build_med,
            "trace_kernel_ms": kern_ms_max,
            "frames_in_flight": br.nbuf,
            "roofline": {
                "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": traffic_src,
                # the same bytes over the steady-state frame interval (launches overlap in flight)
                "achieved_per_step": bytes_launch / (elapsed / args.steps) / 1e9,
                "kernel": TRACE_KERNEL, "bytes_per_launch": bytes_launch,
                "per_ray": {"node_records": float(counters[0]) / (W * H), "tri_tests": float(counters[1]) / (W * H),
                            "hit_frac": float(counters[2]) / (W * H)},
            },
            "cpu_baseline": cpu,
            **extra,
            "host": platform.node(),
        }
        print(json.dumps(out), flush=True)
    br.close()
    cam.destroy()
    scene.destroy()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
