#!/usr/bin/env python3
"""Benchmark: Mrays/s of 1920x1080 primary rays (+ BVH build ms) on 1..8 MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c3|c4|c5|filled] [--no-cpu-baseline]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

Workload (BASELINE.json configs[1] = C2 by default): the Stanford bunny of the reference's
Content/bunny.zip (69,630 triangles, committed as tests/golden/meshes/bunny.npz), camera eye
(-0.34, 1.2, -3.5), setInitialRays(1920, 1080, -16/9, 16/9, -1, 1, 1). A step = one primary-ray
trace of the whole frame with the BVH resident in HBM (inputs resident before the timed region).
--config c3 (armadillo proxy, 278,520 tris, 1080p), c4 (armadillo proxy 3840x2160), c5 (merged
1.1M-tri proxy + one shadow ray per hit) or filled (armadillo proxy, eye close: 85.5 % of pixels hit).

N = 1: frames in flight (--frames-in-flight, default 3): consecutive steps trace into alternating
render targets, each on its own HIP stream (bm_rt_set_stream), so one frame's trace starts while
the previous one drains; `value` is that steady-state rate. The same frame one trace at a time (one
target on the context stream) is reported beside it (`single_frame`), each with its own roofline.

N > 1 (one process per GPU, strong scaling): the SAME fixed frame is cut into 16-row bands dealt
round-robin to the ranks; each rank traces its bands and the C ABI's multi-process context
(bm_options.comm_*, one RCCL communicator in libbeam_hip.so) gathers every plane (packed, triangle
id, t, |n.z|; 16 B/pixel) into rank 0's render target inside the same call. A step = trace + gather.
BM_BENCH_SHARED_DEVICE=1 rehearses N ranks on one GPU (RCCL refuses two ranks on one device): the
bands then travel through torch.distributed over gloo (host memory). Rank 0 checks the assembled
frame against its own single-device trace after the timed region (`frame_check`).

One JSON line on rank 0 (driver contract), with `roofline` (dominant kernel: the trace; achieved =
SURVEY §8(d) algorithmic bytes / kernel time; `hbm_*` = the PMC-measured HBM bytes of the profile
of THIS source revision, see tools/gpu_profile.sh) and `cpu_baseline` (the reference's own
algorithm — kd-tree build + first-hit-leaf march, restated in oracle/ — on the host cores).
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import platform
import re
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)
BAND_H = 16
TRACE_KERNEL = "k_trace_quad<false"  # the timed (non-counting) trace kernel (ray quads, the default variant)
# the kernels of each trace kind (bm_rt_trace_kind), non-counting builds
KIND_KERNELS = {"quads": ("k_trace_quad<false",), "cull+quads": ("k_cull<false", "k_trace_rays<false")}
METRIC = "Mrays/s primary rays @1920x1080 + BVH build ms, 1/2/4/8 MI355X"
# SURVEY §8(d) build bytes per triangle: 12 idx + 36 verts + 8 key/value + P*16 sort + 64 node write
# + 64 refit, with P = 3 one-sweep passes (10-bit digits of the 30-bit Morton key)
BUILD_BYTES_PER_TRI = 12 + 36 + 8 + 3 * 16 + 64 + 64


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="c2", choices=("c2", "c3", "c4", "c5", "filled"))
    ap.add_argument("--leaf-size", type=int, default=4)
    ap.add_argument("--bvh-width", type=int, default=4, choices=(2, 4))
    ap.add_argument("--gather-planes", default="ids", choices=("ids", "packed", "all"),
                    help="N > 1: triangle ids travel and rank 0 rebuilds t, |n.z| and the packed colour "
                         "(4 B/px, every plane exact); 'packed': the reference framebuffer only (4 B/px); "
                         "'all': packed+tri+t+nz as traced (16 B/px)")
    ap.add_argument("--frames-in-flight", type=int, default=3,
                    help="render targets, each on its own HIP stream (1: every frame on the context stream)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extra", action="store_true", help="skip the side figures (other configs, modes)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--only", default="both", choices=("both", "inflight", "single"),
                    help="profiling runs: time only frames in flight or only one frame at a time, so every "
                         "launch rocprofv3 averages is of one kind")
    return ap.parse_args()


def algorithmic_bytes(counters, rays, bvh_width=4):
    """SURVEY.md §8(d) per-ray bytes, with this layout: per node record fetched 64 B (BVH2) or
    112 B (BVH4: six 16-B SoA box planes + refs), 48 B per triangle record tested, 36 B of corner
    normals per hit, 8 B of camera tables per ray (rx, ry), 12 B of output per ray (packed,
    triangle id, t)."""
    nodes, tris, hits = (int(x) for x in counters[:3])
    return (112 if bvh_width == 4 else 64) * nodes + 48 * tris + 36 * hits + (8 + 12) * rays


def shadow_bytes(cnt):
    """Shadow pass (C5): per shadow ray 112 B per BVH4 record + 48 B per triangle test + 1 B out."""
    return 112 * int(cnt[3]) + 48 * int(cnt[4]) + int(cnt[2])


def source_stamp():
    from raytracercuda_amd import build
    return build.source_stamp()


def profile_record(config, kernels=(TRACE_KERNEL,)):
    """PMC record of the trace for `config` from the newest committed profile summary
    (profiles/*_<config>_traffic.json, written by tools/summarize_profile.py from separate
    rocprofv3 --pmc passes of `bench.py --config <config>`) whose source stamp equals this source
    revision's: bytes summed over `kernels` (the launches of one trace), the limiter of the longest.
    (None, reason) when there is none — a profile of other code does not count."""
    files = sorted(glob.glob(os.path.join(REPO, "profiles", f"*_{config}_traffic.json")),
                   key=lambda f: [int(x) for x in re.findall(r"\d+", os.path.basename(f))])
    stamp = source_stamp()
    for f in reversed(files):
        d = json.load(open(f))
        if d.get("stamp") != stamp:
            continue
        recs = [next((v for k, v in d.get("kernels", {}).items() if k.startswith(pre)), None) for pre in kernels]
        if any(r is None for r in recs):
            continue
        out = {"limiter": recs[-1].get("limiter")}
        for key in ("read_bytes_counted", "read_bytes_x2", "write_bytes"):
            vals = [r.get(key) for r in recs]
            out[key] = None if any(v is None for v in vals) else float(sum(vals))
        return out, os.path.relpath(f, REPO)
    return None, f"no profiles/*_{config}_traffic.json of source stamp {stamp} with {', '.join(kernels)}"


def roofline(bytes_launch, kern_ms, step_ms, config, kind="quads", overlapped=False):
    """Roofline of the trace kernel: algorithmic bytes per launch over the launch's duration (HIP
    events on its stream) against the 8 TB/s HBM peak, plus what the counters of this revision's
    profile say: measured HBM bytes (FETCH_SIZE x2 + WRITE_SIZE), L2 hit rate, TA busy."""
    ach = bytes_launch / (kern_ms / 1e3) / 1e9
    kernels = KIND_KERNELS.get(kind, (TRACE_KERNEL,))
    kernel = " + ".join(kernels)
    rec, src = profile_record(config, kernels)
    r = {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": ach / HBM_PEAK_GBS,
         "traffic": None, "traffic_source": src, "kernel": kernel, "bytes_per_launch": bytes_launch,
         "kernel_ms": kern_ms, "achieved_per_step": bytes_launch / (step_ms / 1e3) / 1e9,
         "launch_overlapped": overlapped}
    if rec and rec.get("read_bytes_x2") is not None and rec.get("write_bytes") is not None:
        traffic = float(rec["read_bytes_x2"] + rec["write_bytes"])
        r["traffic"] = traffic
        r["hbm_achieved"] = traffic / (kern_ms / 1e3) / 1e9
        r["hbm_frac"] = r["hbm_achieved"] / HBM_PEAK_GBS
        r["hbm_frac_per_step"] = traffic / (step_ms / 1e3) / 1e9 / HBM_PEAK_GBS
        r["algorithmic_over_hbm_bytes"] = bytes_launch / traffic
    if rec and rec.get("limiter"):
        r["limiter"] = rec["limiter"]
    return r


def cpu_threads():
    """Host threads for the CPU baseline: the cores this process may run on (affinity), capped by
    OMP_NUM_THREADS when set (16 on the gpurun box: the CPU share of one GPU; os.cpu_count() there
    reports the whole machine)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = os.cpu_count() or 1
    cap = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return max(1, min(aff, cap) if cap > 0 else aff), aff


def cpu_baseline(meshes, width, height, cam, eye, orient, seconds, bvh_width=4):
    """The reference's own CPU algorithm (BuildTree.cu:288-306 build, :521-542 march, restated in
    oracle/beam_oracle.c: spatial-median kd-tree over [-30,30]^3 with SAT insertion, first-hit-leaf
    march), timed on T host threads (rows split into 8 ranges per thread; ctypes releases the GIL)
    and on one thread; beside it the scalar LBVH port of this build's GPU algorithm (same math)."""
    from concurrent.futures import ThreadPoolExecutor

    from oracle import Oracle
    o = Oracle()
    err, rays = o.camera_rays(width, height, *cam)
    n = rays.shape[0]
    t0 = time.perf_counter()
    kd = o.kd_build(meshes)
    kd_build_s = time.perf_counter() - t0
    t0 = time.perf_counter()
    bvh = o.bvh_build(meshes, 4, bvh_width)
    bvh_build_s = time.perf_counter() - t0
    T, aff = cpu_threads()

    def run(acc, threads, budget):
        done, el = 0, 0.0
        cuts = np.linspace(0, n, 8 * threads + 1).astype(np.int64)
        with ThreadPoolExecutor(max_workers=threads) as pool:
            while el < budget:
                t0 = time.perf_counter()
                list(pool.map(lambda k: acc.render(rays, eye, orient, int(cuts[k]), int(cuts[k + 1])),
                              range(len(cuts) - 1)))
                el += time.perf_counter() - t0
                done += n
        return done, el

    kT, keT = run(kd, T, seconds * 0.5)
    k1, ke1 = run(kd, 1, seconds * 0.25)
    bT, beT = run(bvh, T, seconds * 0.25)
    cpu = "unknown"
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                cpu = ln.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"value": kT / keT / 1e6, "unit": "Mrays/s", "cores": T, "kind": "port",
            "sample": f"the reference's kd-tree march (oracle restatement of BuildTree.cu:367-499): {kT // n} full "
                      f"{width}x{height} frames ({kT} rays, {keT:.1f} s) on {T} threads (rows split 8 ranges/thread) "
                      f"+ {k1 // n} frames on 1 thread ({ke1:.1f} s); kd build {kd_build_s * 1e3:.0f} ms (1 thread)",
            "single_thread_mrays_s": k1 / ke1 / 1e6, "build_ms": kd_build_s * 1e3,
            "threads_note": f"{T} threads = min(affinity {aff}, OMP_NUM_THREADS)",
            "affinity_cpus": aff, "cpu_model": cpu, "host_threads": os.cpu_count(),
            "lbvh_port": {"mrays_s": bT / beT / 1e6, "threads": T, "build_ms": bvh_build_s * 1e3,
                          "note": "scalar LBVH of oracle/ (this build's GPU algorithm, same arithmetic)"}}


def hits_of(packed):
    return int((packed != 0x0000FF00).sum())


class Workload:
    """One config on one device: scene (built), camera, counters and their algorithmic bytes."""

    def __init__(self, ctx, name, torch, stream):
        from raytracercuda_amd import beam, scenes
        self.beam, self.scenes, self.torch, self.stream = beam, scenes, torch, stream
        self.ctx, self.name = ctx, name
        c = scenes.CONFIGS[name]
        self.cfg = c
        self.W, self.H, self.eye, self.light = c["width"], c["height"], c["eye"], c["light"]
        self.orient = scenes.IDENTITY
        self.meshes = scenes.scene(c["scene"])
        self.scene = beam.IScene.create(ctx)
        self.keep = beam.upload_meshes(ctx, self.scene, self.meshes)
        builds = [self.scene.updateGPUScene(stats=True)["build_ms"] for _ in range(7)]
        self.build_ms = float(np.median(builds[2:]))
        self.st = self.scene.last_stats
        self.cam = beam.ICamera.create(ctx)
        ctx._check(self.cam.setInitialRays(self.W, self.H, *c["rays"]))
        rt = beam.IRenderTarget.createOffscreen(ctx, self.W, self.H)
        if self.light:
            self.counters = self.cam.traceShadowCounters(self.eye, self.orient, self.scene, rt, self.light)
        else:
            self.counters = self.cam.traceCounters(self.eye, self.orient, self.scene, rt)
        rt.destroy()
        self.rays = self.W * self.H
        self.bytes = algorithmic_bytes(self.counters, self.rays, self.st["bvh_width"])
        if self.light:
            self.bytes += shadow_bytes(self.counters)

    def trace(self, rt):
        if self.light:
            return self.cam.traceShadow(self.eye, self.orient, self.scene, rt, self.light)
        return self.cam.trace(self.eye, self.orient, self.scene, rt)

    def run(self, nbuf, steps, warmup):
        """Trace `steps` frames into nbuf targets (own streams when nbuf > 1). Returns (ms per
        step from the host clock between synchronisations, mean per-launch ms from HIP events on
        each launch's stream, the last target's planes)."""
        torch, beam = self.torch, self.beam
        rts = [beam.IRenderTarget.createOffscreen(self.ctx, self.W, self.H) for _ in range(nbuf)]
        streams = [torch.cuda.Stream() for _ in range(nbuf)] if nbuf > 1 else [None]
        for rt, s in zip(rts, streams):
            if s is not None:
                rt.setStream(s.cuda_stream)
        for i in range(warmup):
            self.ctx._check(self.trace(rts[i % nbuf]))
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
        self.ctx.sync()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(steps):
            s = streams[i % nbuf] or self.stream
            ev[i][0].record(s)
            self.ctx._check(self.trace(rts[i % nbuf]))
            ev[i][1].record(s)
        self.ctx.sync()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        kern = float(np.mean([a.elapsed_time(b) for a, b in ev]))
        last = rts[(steps - 1) % nbuf].read(rgb=True)
        self.kind = rts[(steps - 1) % nbuf].traceKind()
        if self.light:
            last["shadow"] = rts[(steps - 1) % nbuf].readShadow()
        for rt in rts:
            rt.destroy()
        return el / steps * 1e3, kern, last

    def reference_frame(self):
        rt = self.beam.IRenderTarget.createOffscreen(self.ctx, self.W, self.H)
        self.ctx._check(self.trace(rt))
        f = rt.read(rgb=True)
        if self.light:
            f["shadow"] = rt.readShadow()
        rt.destroy()
        return f

    def per_ray(self):
        r = {"node_records": float(self.counters[0]) / self.rays, "tri_tests": float(self.counters[1]) / self.rays,
             "hit_frac": float(self.counters[2]) / self.rays}
        if self.light:
            r["shadow_rays"] = int(self.counters[2])
            r["shadow_node_records_per_shadow_ray"] = float(self.counters[3]) / max(int(self.counters[2]), 1)
            r["shadow_tri_tests_per_shadow_ray"] = float(self.counters[4]) / max(int(self.counters[2]), 1)
        return r

    def measure(self, nbuf, steps, warmup, only="both"):
        """Frames in flight and one frame at a time, each with its roofline, and the in-flight frame
        checked bit for bit against a trace on the context stream. only="inflight"/"single" (profiling
        runs) times one of the two and reports it in both places."""
        if only == "single":
            nbuf = 1
        step_ms, kern_ms, last = self.run(nbuf, steps, warmup)
        kind = self.kind
        if only == "both":
            ref = self.reference_frame()
            check = all(np.array_equal(last[k], ref[k]) for k in ref)
        else:
            # profiling runs (tools/gpu_profile.sh) trace nothing but the timed frames, so the rocprof
            # summary's per-kernel average is the timed launches' (under rocprofv3 the untimed
            # reference frame into a fresh target took ~28 ms and dominated that average)
            ref, check = last, None
        s_kind = kind
        if not (only != "both" or nbuf == 1):
            s_step, s_kern = self.run(1, steps, warmup)[:2]
            s_kind = self.kind
        else:
            s_step, s_kern = step_ms, kern_ms
        out = {"scene": self.cfg["scene"], "tris": self.st["num_tris"], "width": self.W, "height": self.H,
               "eye": list(self.eye), "build_ms": self.build_ms,
               "build_roofline": build_roofline(self.st["num_tris"], self.build_ms),
               "frames_in_flight": nbuf, "mrays_s": self.rays / (step_ms / 1e3) / 1e6, "ms_per_step": step_ms,
               "trace_kernel_ms": kern_ms, "frame_hits": hits_of(ref["packed"]), "frame_check": None if check is None else bool(check),
               "trace_kind": kind,
               "roofline": roofline(self.bytes, kern_ms, step_ms, self.name, kind, overlapped=nbuf > 1),
               "single_frame": None if only == "inflight" else
               {"mrays_s": self.rays / (s_step / 1e3) / 1e6, "ms_per_step": s_step, "trace_kernel_ms": s_kern,
                "trace_kind": s_kind, "roofline": roofline(self.bytes, s_kern, s_step, self.name, s_kind)},
               "per_ray": self.per_ray()}
        if self.light:
            out["light"] = list(self.light)
            out["shadowed"] = int(self.counters[5])
            out["rays_incl_shadow_per_s_M"] = (self.rays + int(self.counters[2])) / (step_ms / 1e3) / 1e6
        return out

    def close(self):
        self.cam.destroy()
        self.scene.destroy()
        self.keep = None


def build_roofline(ntris, build_ms):
    b = ntris * BUILD_BYTES_PER_TRI
    ach = b / (build_ms / 1e3) / 1e9
    return {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": ach / HBM_PEAK_GBS,
            "bytes": b, "bytes_per_tri": BUILD_BYTES_PER_TRI,
            "note": "SURVEY §8(d) B_tri with P = 3 sort passes; build_ms = device time of all build launches"}


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
    reps = 10 if mode == "kd" else 3
    ea.record(stream)
    for _ in range(reps):
        ctx._check(cam.trace(eye, orient, sc, rt))
    eb.record(stream)
    torch.cuda.synchronize()
    ms = ea.elapsed_time(eb) / reps
    st = sc.kdStats() if mode == "kd" else sc.gridStats()
    hits = hits_of(rt.read(tri_id=False, t=False)["packed"])
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


def single_gpu(args, torch, stream):
    from raytracercuda_amd import beam, scenes
    ctx = beam.Context(device=0, stream=stream.cuda_stream, leaf_size=args.leaf_size, bvh_width=args.bvh_width)
    wl = Workload(ctx, args.config, torch, stream)
    nbuf = max(1, args.frames_in_flight)
    head = wl.measure(nbuf, args.steps, args.warmup, args.only)
    extra = {}
    if not args.no_extra:
        for name in ("c3", "filled", "c5"):
            if name == args.config:
                continue
            w2 = Workload(ctx, name, torch, stream)
            extra[{"c3": "c3_armadillo_proxy", "filled": "filled_view", "c5": "c5_merged_proxy_shadow"}[name]] = \
                w2.measure(nbuf, max(10, args.steps // 2), args.warmup)
            w2.close()
        c = scenes.CONFIGS[args.config]
        extra["reference_mode"] = reference_side_figure(0, stream, wl.meshes, wl.W, wl.H, c["rays"], wl.eye,
                                                        wl.orient)
        extra["hashed_grid"] = reference_side_figure(0, stream, wl.meshes, wl.W, wl.H, c["rays"], wl.eye,
                                                     wl.orient, "hash")
    cpu = None
    if not args.no_cpu_baseline:
        c = scenes.CONFIGS[args.config]
        cpu = cpu_baseline(wl.meshes, wl.W, wl.H, c["rays"], wl.eye, wl.orient, args.cpu_seconds,
                           wl.st["bvh_width"])
    wl.close()
    ctx.close()
    return head, extra, cpu


def multi_gpu(args, torch, dist, rank, world, local, shared):
    """Strong scaling of the fixed frame over `world` processes; returns rank 0's record."""
    from raytracercuda_amd import beam, multigpu, scenes
    dev = torch.device("cuda", local)
    stream = torch.cuda.current_stream()
    c = scenes.CONFIGS[args.config]
    W, H, eye, orient, light = c["width"], c["height"], c["eye"], scenes.IDENTITY, c["light"]
    planes = {"ids": None, "packed": ["packed"], "all": ["packed", "tri_id", "t", "nz"]}[args.gather_planes]
    torch_gather = shared
    ctx, transport = None, None
    if not shared:
        # the C ABI's own RCCL communicator; every rank must end up on the same transport, so a
        # failure anywhere (no librccl, init error) moves all ranks to the torch.distributed gather
        err = ""
        try:
            obj = [beam.comm_unique_id() if rank == 0 else None]
            dist.broadcast_object_list(obj, src=0)
            ctx = beam.Context(device=local, stream=stream.cuda_stream, leaf_size=args.leaf_size,
                               comm=(rank, world, obj[0]), planes=planes)
        except beam.BeamError as e:  # reported in the line, not hidden
            err = str(e)
        ok = torch.tensor([0 if ctx is None else 1], dtype=torch.int32, device=dev)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        if int(ok[0]) == 1:
            transport = "RCCL send/recv inside libbeam_hip.so (bm_options.comm_*), xGMI"
        else:
            if ctx is not None:
                ctx.close()
            ctx = None
            torch_gather = True
            transport = ("torch.distributed gather over RCCL (the C-ABI communicator failed to start: "
                         f"{err or 'on another rank'})")
    if torch_gather:
        ctx = beam.Context(device=local, stream=stream.cuda_stream, leaf_size=args.leaf_size)
        if shared:
            transport = "torch.distributed gather over gloo (shared-device rehearsal: all ranks on one GPU)"
    meshes = scenes.scene(c["scene"])
    scene = beam.IScene.create(ctx)
    keep = beam.upload_meshes(ctx, scene, meshes)
    builds = [scene.updateGPUScene(stats=True)["build_ms"] for _ in range(7)]
    st = scene.last_stats
    cam = beam.ICamera.create(ctx)
    ctx._check(cam.setInitialRays(W, H, *c["rays"]))
    nbuf = max(2, args.frames_in_flight)
    if torch_gather:
        br = multigpu.BandRenderer(ctx, scene, cam, W, H, BAND_H, rank, world, dev,
                                   planes="packed" if args.gather_planes == "packed" else "full",
                                   frames_in_flight=nbuf)

        def step(i):
            br.acquire()
            ctx._check(br.trace(eye, orient, light))
            br.gather()
    else:
        rts = [beam.IRenderTarget.createOffscreen(ctx, W, H) for _ in range(nbuf)]
        streams = [torch.cuda.Stream(device=dev) for _ in range(nbuf)]
        for rt, s in zip(rts, streams):
            rt.setStream(s.cuda_stream)

        def step(i):
            if light:
                ctx._check(cam.traceShadow(eye, orient, scene, rts[i % nbuf], light))
            else:
                ctx._check(cam.trace(eye, orient, scene, rts[i % nbuf]))
    for i in range(args.warmup):
        step(i)
    ctx.sync()
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i)
    ctx.sync()
    torch.cuda.synchronize()
    dist.barrier()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64, device="cpu" if shared else dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t[0])
    out = None
    if rank == 0:
        one = beam.Context(device=local)  # the same frame traced by this GPU alone
        s1 = beam.IScene.create(one)
        k1 = beam.upload_meshes(one, s1, meshes)
        s1.updateGPUScene()
        c1 = beam.ICamera.create(one)
        one._check(c1.setInitialRays(W, H, *c["rays"]))
        r1 = beam.IRenderTarget.createOffscreen(one, W, H)
        cnt = c1.traceCounters(eye, orient, s1, r1)  # traversal counters of the whole frame (writes it too)
        if light:
            one._check(c1.traceShadow(eye, orient, s1, r1, light))
        full = r1.read(rgb=True)
        if light:
            full["shadow"] = r1.readShadow()
        if torch_gather:
            fr = br.frame().cpu().numpy()
            got = {"packed": fr[0].view(np.uint32)}
            if fr.shape[0] == 3:
                got.update(tri_id=fr[1].view(np.uint32), t=fr[2].view(np.float32))
        else:
            last = rts[(args.steps - 1) % nbuf]
            got = last.read(rgb=args.gather_planes != "packed")
            if args.gather_planes == "packed":
                got = {"packed": got["packed"]}
            elif light:
                got["shadow"] = last.readShadow()
        check = all(np.array_equal(got[k], full[k]) for k in got)
        for h in (r1, c1, s1):
            h.destroy()
        del k1
        one.close()
        out = {"elapsed": elapsed, "W": W, "H": H, "transport": transport, "frame_check": bool(check),
               "checked_planes": sorted(got), "build_ms": float(np.median(builds[2:])), "tris": st["num_tris"],
               "frame_hits": hits_of(full["packed"]), "nbuf": nbuf, "scene": c["scene"], "eye": list(eye),
               "frame_bytes": algorithmic_bytes(cnt, W * H, st["bvh_width"])}
    if torch_gather:
        br.close()
    else:
        for rt in rts:
            rt.destroy()
    cam.destroy()
    scene.destroy()
    del keep
    ctx.close()
    return out


def main():
    args = parse()
    import torch
    import torch.distributed as dist

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
    if world > 1:
        if shared:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    from raytracercuda_amd import scenes
    c = scenes.CONFIGS[args.config]
    common = {"metric": METRIC, "unit": "Mrays/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
              "higher_is_better": True, "vs_baseline": None, "dtype": "f32",
              "data": f"synthetic pinhole camera rays over {c['scene']} (reference Content/bunny.zip; proxies per "
                      f"SURVEY §8(d))", "source_stamp": source_stamp()}
    if world == 1:
        stream = torch.cuda.current_stream()
        head, extra, cpu = single_gpu(args, torch, stream)
        out = {**common, "value": head["mrays_s"], "ms_per_step": head["ms_per_step"], "scaling": "strong",
               "config": {"workload": f"{args.config}: {head['scene']} ({head['tris']} tris) {head['width']}x"
                                      f"{head['height']} primary rays{' + shadow rays' if c['light'] else ''}, "
                                      f"{head['frames_in_flight']} frames in flight (one HIP stream per render "
                                      f"target)",
                          "config_id": args.config, "scene": head["scene"], "tris": head["tris"],
                          "width": head["width"], "height": head["height"], "leaf_size": args.leaf_size,
                          "bvh_width": args.bvh_width, "parallelism": "1 GPU"},
               "build_ms": head["build_ms"], "build_roofline": head["build_roofline"], "trace_kind": head["trace_kind"],
               "trace_kernel_ms": head["trace_kernel_ms"], "frames_in_flight": head["frames_in_flight"],
               "roofline": head["roofline"], "single_frame": head["single_frame"], "per_ray": head["per_ray"],
               "frame_hits": head["frame_hits"], "frame_check": head["frame_check"], "cpu_baseline": cpu,
               **extra, "host": platform.node()}
        print(json.dumps(out), flush=True)
        return
    rec = multi_gpu(args, torch, dist, rank, world, local, shared)
    if rank == 0:
        rays = rec["W"] * rec["H"]
        value = rays * args.steps / rec["elapsed"] / 1e6
        out = {**common, "value": value, "ms_per_step": rec["elapsed"] / args.steps * 1e3, "scaling": "strong",
               "config": {"workload": f"{args.config}: {rec['scene']} ({rec['tris']} tris), one fixed {rec['W']}x"
                                      f"{rec['H']} frame, {BAND_H}-row bands round-robin over {world} GPUs, "
                                      f"gather of every band into rank 0 per step: {rec['transport']}; "
                                      f"{rec['nbuf']} frames in flight",
                          "config_id": args.config, "scene": rec["scene"], "tris": rec["tris"],
                          "width": rec["W"], "height": rec["H"], "band_h": BAND_H,
                          "gather_planes": args.gather_planes, "parallelism": f"screen-bands x{world}"},
               "build_ms": rec["build_ms"], "frame_check": rec["frame_check"],
               "checked_planes": rec["checked_planes"], "frame_hits": rec["frame_hits"],
               "gather_bytes_per_frame": rays * (16 if args.gather_planes == "all" else 4) * (world - 1) // world,
               "roofline": roofline(rec["frame_bytes"] / world, rec["elapsed"] / args.steps * 1e3,
                                    rec["elapsed"] / args.steps * 1e3, args.config, "cull+quads", overlapped=True),
               "roofline_note": "per rank: its share of the frame's algorithmic bytes over the step time "
                                "(trace + gather, frames in flight); no per-kernel split at N > 1",
               "cpu_baseline": None, "host": platform.node()}
        print(json.dumps(out), flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
