#!/usr/bin/env python3
"""Benchmark: Mrays/s of 1920x1080 primary rays (+ BVH build ms) on 1..8 MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c3|c4|c5|filled] [--no-cpu-baseline]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

Workload: BASELINE.json's own configs. N = 1 (default): C3 = configs[2], north_star's target config
— the armadillo proxy (armadillo.obj is absent from the reference, .MISSING_LARGE_BLOBS:3-8; SURVEY
§8(d): the bunny of Content/bunny.zip subdivided once, 278,520 triangles) at 1920x1080, camera eye
(-0.34, 1.2, -3.5), setInitialRays(1920, 1080, -16/9, 16/9, -1, 1, 1). N > 1 (default): C4 =
configs[3], the same proxy at 3840x2160, which BASELINE names for 2/4/8 GPUs; the N = 1 line carries
C4's one-GPU figure (`c4_armadillo_4k`) as the curve's first point, beside C2 (bunny 1080p),
the filled view and C5 (merged 1.1M-triangle proxy + shadow rays). A step = one primary-ray trace of
the whole frame with the BVH resident in HBM (inputs resident before the timed region).
--config picks another workload for `value`.

N = 1: frames in flight (--frames-in-flight, default 3): consecutive steps trace into alternating
render targets, each on its own HIP stream (bm_rt_set_stream), so one frame's trace starts while
the previous one drains; `value` is that steady-state rate. The same frame one trace at a time (one
target on the context stream) is reported beside it (`single_frame`), each with its own roofline.

N > 1 (one process per GPU, strong scaling): the SAME fixed frame is cut into 16-row bands dealt
round-robin to the ranks; each rank traces its bands and the C ABI's multi-process context
(bm_context_start_comm, one RCCL communicator in libbeam_hip.so) gathers the triangle-id plane
(4 B/pixel; rank 0 rebuilds t, |n.z| and the packed colour from it) into rank 0's render target
inside the same call. A step = trace + gather; `trace_ms` / `gather_ms` split it (HIP events around
each rank's band trace and the exchange after it, bm_rt_last_timing).
BM_BENCH_SHARED_DEVICE=1 rehearses N ranks on one GPU (RCCL refuses two ranks on one device): the
bands then travel through torch.distributed over gloo (host memory). Rank 0 checks the assembled
frame against its own single-device trace after the timed region (`frame_check`).

One JSON line on rank 0 (driver contract), with `roofline` (dominant kernel: the trace) and
`cpu_baseline` (the reference's own algorithm — kd-tree build + first-hit-leaf march, restated in
oracle/ — on the host cores). Roofline fields:
* `traffic` = HBM bytes per launch (one frame) from PMC counters measured LIVE on this run's code (N = 1:
  before anything touches the GPU, bench.py re-runs itself under `rocprofv3 --pmc` once per counter
  group, tools/pmc.py; FETCH_SIZE x2 per the gfx950 note + WRITE_SIZE); `kernel_ms` = the time basis: the
  launch's duration one frame at a time (HIP events on its stream), the step time with frames in flight
  (their launches overlap); `achieved` = traffic / kernel_ms, `frac` = achieved / 8 TB/s;
* `bound` = the limiter the counters measure ("latency": waves mostly parked on s_waitcnt; "issue";
  "hbm" only when the counters put the kernel near the HBM roofline), details in `limiter`;
* `levels.data` = SURVEY §8(d)'s algorithmic bytes per launch (every node record, triangle record, normal
  and output the traversal touches, almost all served by L1/L2/MALL) over the same basis, against the
  aggregate L2 peak (they are not HBM bytes); `levels.l2` = counted L1->L2 request bytes.
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
L2_PEAK_GBS = 34500.0  # aggregate L2 (8 XCDs x 4 MiB), MI355X_MICROARCH.md §L2
BAND_H = 16
TRACE_KERNEL = "k_trace_quad<false"  # the timed (non-counting) trace kernel (ray quads, the default variant)
# the kernels of each trace kind (bm_rt_trace_kind), non-counting builds
KIND_KERNELS = {"quads": ("k_trace_quad<false",), "cull+quads": ("k_cull<false", "k_trace_rays<false"),
                "lanes": ("k_trace_persistent<false",), "kd march": ("k_kd_march_coop<false",),
                "packets": ("k_trace_packet<",)}
PMC_STEPS, PMC_WARMUP = 10, 3  # launches per segment in the counter passes
METRIC = "Mrays/s primary rays @1920x1080 + BVH build ms, 1/2/4/8 MI355X"
# SURVEY §8(d) build bytes per triangle: 12 idx + 36 verts + 8 key/value + P*16 sort + 64 node write
# + 64 refit, with P = 3 one-sweep passes (10-bit digits of the 30-bit Morton key)
BUILD_BYTES_PER_TRI = 12 + 36 + 8 + 3 * 16 + 64 + 64
SIDE_STEPS, SIDE_WARMUP = 60, 6  # side figures (other configs): timed frames and warm-up, independent of --steps
# frames in flight: the launch-duration events bracket every EV_EVERY-th frame (a pair around every frame
# cost 2-5 % of the in-flight rate: tools/host_rate.py); one frame at a time: every frame
EV_EVERY = 4
FULL_RECORD = os.path.join("gpurun_out", "bench_full.json")  # the uncompacted N = 1 record (named in the line)
BENCH_PARAMS = {}  # --param name=value (A/B runs only): tuning parameters of every context this script makes


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="auto", choices=("auto", "c2", "c3", "c4", "c5", "filled"),
                    help="auto: c3 at N = 1 (north_star's armadillo 1080p), c4 (armadillo 4K) at N > 1")
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
    ap.add_argument("--pmc", default="auto", choices=("auto", "on", "off"),
                    help="live PMC counter passes (rocprofv3 --pmc children of this script) for roofline.traffic; "
                         "auto = N = 1 and not already under a profiler")
    ap.add_argument("--pmc-keep", default=None, help="copy the counter passes' CSVs and logs into this directory")
    ap.add_argument("--pmc-child", default=None, help=argparse.SUPPRESS)  # internal: one counter pass
    ap.add_argument("--param", action="append", default=[], metavar="NAME=VALUE",
                    help="A/B only: a tuning parameter (bm_context_set_param, raytracercuda_amd/_lib.py PARAMS) of "
                         "every context; the defaults are the library's measured-best settings")
    args = ap.parse_args()
    for kv in args.param:
        k, v = kv.split("=", 1)
        BENCH_PARAMS[k] = int(v)
    return args


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


def committed_profile(config, kernels=(TRACE_KERNEL,)):
    """Fallback when no live counters exist (e.g. --pmc off): the newest committed profile summary
    (profiles/*_<config>_traffic.json, tools/summarize_profile.py) whose source stamp equals this
    source revision's — a profile of other code does not count. (record, source) or (None, reason)."""
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
        out = {"limiter": {k: v for k, v in (recs[-1].get("limiter") or {}).items()
                           if k in ("l2_hit", "ta_busy", "wave_time_issue_stalled", "wave_time_issuing")}}
        lim = recs[-1].get("limiter") or {}
        if "wave_time_waiting_on_loads_or_barrier" in lim:
            out["limiter"]["wave_time_waiting_on_loads"] = lim["wave_time_waiting_on_loads_or_barrier"]
        for key in ("read_bytes_counted", "read_bytes_x2", "write_bytes"):
            vals = [r.get(key) for r in recs]
            out[key] = None if any(v is None for v in vals) else float(sum(vals))
        out["traffic"] = (None if out["read_bytes_x2"] is None or out["write_bytes"] is None
                          else out["read_bytes_x2"] + out["write_bytes"])
        return out, os.path.relpath(f, REPO)
    return None, f"no profiles/*_{config}_traffic.json of source stamp {stamp} with {', '.join(kernels)}"


def pmc_segment(pmc, label, config, kernels):
    """The counter record of one measured segment: live (this run's passes) or a committed profile of
    this source revision; (record or None, source)."""
    if pmc is not None:
        rec = pmc["segments"].get(label)
        if rec is not None and rec.get("traffic") is not None:
            return rec, "live rocprofv3 --pmc passes of this run (tools/pmc.py)"
        err = "; ".join(f"{k}: {v}" for k, v in pmc.get("errors", {}).items()) or "segment missing"
        committed, src = committed_profile(config, kernels)
        if committed:
            return committed, src + f" (live counters unusable: {err})"
        return None, f"live counters unusable ({err}); {src}"
    return committed_profile(config, kernels)


def roofline(bytes_launch, kern_ms, step_ms, rec, src, kernels, overlapped=False):
    """Roofline of the trace (every byte count against the peak of the level that serves it,
    over a time that lies inside the step).

    Time basis `kernel_ms`: one launch at a time (overlapped False) = the launch's average duration (HIP
    events on its stream), which lies inside the step (kernel_ms <= step_ms). Frames in flight (overlapped
    True): consecutive launches overlap (each spans ~2.5 steps), so a launch's duration is not the GPU time
    one frame costs; the basis is the step itself (kernel_ms = step_ms, the launch span stays in `launch_ms`).

    Contract fields: `traffic` = HBM bytes of one launch (= one frame) from the PMC counters (FETCH_SIZE x2
    per the gfx950 note + WRITE_SIZE), `achieved` = traffic / kernel_ms, `peak` = the 8 TB/s HBM peak, `frac`
    (null without counters). The SURVEY §8(d) algorithmic bytes (every node/triangle record the traversal
    touches, ~90 % served by L1/L2/MALL) go only under `levels.data`, against the ~34.5 TB/s aggregate L2
    peak; `levels.l2` = counted L1->L2 request bytes (TCP_TCC_READ/WRITE_REQ x 128 / 64 B, calibrated,
    tools/l2_calib.py) against the same peak; `levels.hbm` = the contract fields. `bound` = the limiter the
    counters measure ("hbm"/"l2" only when that level runs near its peak, else "latency" or "issue" from the
    wave-time split, `limiter`)."""
    from tools import pmc as tpmc
    basis = step_ms if overlapped else kern_ms
    gbs = lambda b: b / (basis / 1e3) / 1e9  # noqa: E731
    r = {"bound": None, "achieved": None, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": None, "traffic": None,
         "kernel": " + ".join(kernels), "kernel_ms": basis, "step_ms": step_ms, "launch_ms": kern_ms,
         "launch_overlapped": overlapped, "bytes_per_launch": bytes_launch, "traffic_source": src,
         "basis": ("frames in flight: one frame's bytes per step (launches of consecutive frames overlap; "
                   f"launch_ms = HIP events around every {EV_EVERY}th launch)") if overlapped else
                  "one launch at a time: bytes per launch over its duration (HIP events around every launch)"}
    levels = {}
    if bytes_launch:
        levels["data"] = {"bytes": bytes_launch, "achieved": gbs(bytes_launch), "peak": L2_PEAK_GBS,
                          "frac": gbs(bytes_launch) / L2_PEAK_GBS}
    lim = (rec or {}).get("limiter") or {}
    if rec and rec.get("traffic") is not None:
        traffic = float(rec["traffic"])
        a = gbs(traffic)
        r.update(traffic=traffic, achieved=a, frac=a / HBM_PEAK_GBS)
        levels["hbm"] = {"bytes": traffic, "read_x2": rec.get("read_bytes_x2"), "write": rec.get("write_bytes"),
                         "achieved": a, "peak": HBM_PEAK_GBS, "frac": a / HBM_PEAK_GBS}
    if rec and rec.get("l2_bytes") is not None:
        l2 = float(rec["l2_bytes"])
        levels["l2"] = {"bytes": l2, "read": rec.get("l2_read_bytes"), "write": rec.get("l2_write_bytes"),
                        "achieved": gbs(l2), "peak": L2_PEAK_GBS, "frac": gbs(l2) / L2_PEAK_GBS}
    r["levels"] = levels
    if lim:
        r["limiter"] = lim
    r["bound"] = tpmc.bound_of(lim, levels.get("hbm", {}).get("frac"), levels.get("l2", {}).get("frac"))
    if rec and rec.get("resources"):
        r["resources"] = rec["resources"]
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
            "algorithm": "reference",
            "algorithm_note": "the reference's own algorithm (kd-tree build + first-hit-leaf march, "
                              "BuildTree.cu:154-306, 367-499), restated in plain C in oracle/beam_oracle.c; kind "
                              "'port' = the oracle's restatement, not a compiled reference (the reference's CPU path "
                              "needs a stand-in cuda_runtime.h, which this build may not write: DESIGN §3)",
            "sample": f"the reference's kd-tree march (oracle restatement of BuildTree.cu:367-499): {kT // n} full "
                      f"{width}x{height} frames ({kT} rays, {keT:.1f} s) on {T} threads (rows split 8 ranges/thread) "
                      f"+ {k1 // n} frames on 1 thread ({ke1:.1f} s); kd build {kd_build_s * 1e3:.0f} ms (1 thread)",
            "single_thread_mrays_s": k1 / ke1 / 1e6, "build_ms": kd_build_s * 1e3,
            "threads_note": f"{T} threads = min(affinity {aff}, OMP_NUM_THREADS): the host CPU share of one GPU "
                            f"on the GPU box (its rules size worker pools to that share); the affinity mask lists all "
                            f"{aff} CPUs of the machine, shared with the other GPUs' jobs, so an all-affinity run is "
                            f"not made; single_thread_mrays_s x {aff} would be the linear-scaling bound",
            "all_affinity_linear_bound_mrays_s": k1 / ke1 / 1e6 * aff,
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
        self.nverts = sum(int(np.asarray(m["pos"]).reshape(-1, 3).shape[0]) for m in self.meshes)
        # the BVH4 records a traversal can reach (the product's part of the records the build writes)
        self.reachable = len(beam.reachable_records(self.scene.export()[0])) if self.st["bvh_width"] == 4 else None
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
        every = EV_EVERY if nbuf > 1 else 1
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
        self.ctx.sync()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(steps):
            s = streams[i % nbuf] or self.stream
            if i % every == 0:
                ev[i][0].record(s)
            self.ctx._check(self.trace(rts[i % nbuf]))
            if i % every == 0:
                ev[i][1].record(s)
        self.ctx.sync()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        kern = float(np.mean([a.elapsed_time(b) for i, (a, b) in enumerate(ev) if i % every == 0]))
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

    def measure(self, nbuf, steps, warmup, only="both", pmc=None):
        """Frames in flight and one frame at a time, each with its roofline, and the in-flight frame
        checked bit for bit against a trace on the context stream. only="inflight"/"single" (profiling
        runs) times one of the two and reports it in both places. pmc: the live counter summary
        (segments "<config>/inflight", "<config>/single")."""
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
        ks, s_ks = KIND_KERNELS.get(kind, (TRACE_KERNEL,)), KIND_KERNELS.get(s_kind, (TRACE_KERNEL,))
        rec, src = pmc_segment(pmc, f"{self.name}/{'inflight' if nbuf > 1 else 'single'}", self.name, ks)
        s_rec, s_src = pmc_segment(pmc, f"{self.name}/single", self.name, s_ks)
        out = {"scene": self.cfg["scene"], "tris": self.st["num_tris"], "width": self.W, "height": self.H,
               "eye": list(self.eye), "build_ms": self.build_ms,
               "build_roofline": build_roofline(self.st["num_tris"], self.build_ms,
                                                (pmc or {}).get("builds", {}).get(self.name), self.nverts,
                                                self.reachable, "lsd" if self.st["sort_path"] == 1 else "msd"),
               "frames_in_flight": nbuf, "mrays_s": self.rays / (step_ms / 1e3) / 1e6, "ms_per_step": step_ms,
               "trace_kernel_ms": kern_ms, "frame_hits": hits_of(ref["packed"]), "frame_check": None if check is None else bool(check),
               "trace_kind": kind,
               "roofline": roofline(self.bytes, kern_ms, step_ms, rec, src, ks, overlapped=nbuf > 1),
               "single_frame": None if only == "inflight" else
               {"mrays_s": self.rays / (s_step / 1e3) / 1e6, "ms_per_step": s_step, "trace_kernel_ms": s_kern,
                "trace_kind": s_kind, "roofline": roofline(self.bytes, s_kern, s_step, s_rec, s_src, s_ks)},
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


def build_required(ntris, nverts, nrec, sort="msd"):
    """the HBM bytes each build kernel must move, every datum once, for what the product
    needs — n triangles, V vertices, R reachable BVH4 records (128 B). The top-digit-first sort
    (2^14..2^22 triangles) is k_onesweep_wide once + k_bucket_sort; the three-pass LSD sort is three
    k_onesweep_wide passes.
      k_gather         indices 12n + positions 12V in, AABB centres 12n out (Morton input)
      k_morton         centres 12n in, (key, index) 8n out
      k_onesweep_wide  (key, index) 8n in + 8n out per pass; on the top-digit path its extra workgroups
                       also gather the corner normals: indices 12n + normals 12V in, 36n out
      k_bucket_sort    8n in + 8n out
      k_span_chunk     sorted keys 4n + permutation 4n + indices 12n + positions 12V in; the sorted
                       triangle records 48n and the chunk-local BVH4 records (~R x 128) out
      k_chunk_table*, k_pack4_*  chunk unions and the spanning nodes' records: O(n / 512), counted as 0
    """
    n, V, R = float(ntris), float(nverts), float(nrec)
    msd = sort == "msd"
    req = {"k_gather": 12 * n + 12 * V + 12 * n,
           "k_morton": 12 * n + 8 * n,
           "k_onesweep_wide": (16 * n + (12 * n + 12 * V + 36 * n)) if msd else 3 * 16 * n + (12 * n + 12 * V + 36 * n),
           "k_bucket_sort": 16 * n if msd else 0.0,
           "k_span_chunk": 4 * n + 4 * n + 12 * n + 12 * V + 48 * n + 128 * R}
    return {k: v for k, v in req.items() if v > 0}


def build_roofline(ntris, build_ms, rec=None, nverts=None, nrec=None, sort="msd"):
    """The build's roofline: the HBM bytes the product needs per build (build_required, per kernel: the
    sorted triangle records and corner normals included) over the build's device time, against the HBM
    peak; the PMC-counted HBM bytes per build (sum over its launches) and, per kernel, counted / required.
    SURVEY §8(d)'s B_tri model (232 B/tri, P = 3 sort passes) stays beside it (`model_bytes`)."""
    model = ntris * BUILD_BYTES_PER_TRI
    req = build_required(ntris, nverts, nrec, sort) if nverts is not None and nrec is not None else None
    b = sum(req.values()) if req else model
    ach = b / (build_ms / 1e3) / 1e9
    r = {"bound": "latency", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": ach / HBM_PEAK_GBS,
         "bytes": b, "bytes_per_tri": b / max(ntris, 1), "model_bytes": model, "model_bytes_per_tri": BUILD_BYTES_PER_TRI,
         "traffic": None,
         "note": ("achieved = the per-kernel required bytes (build_required) over build_ms (device time of all build "
                  "launches)" if req else "achieved = SURVEY §8(d) B_tri with P = 3 sort passes over build_ms") +
                 "; bound: dependent launches and look-back chains at small n (DESIGN §4), not HBM"}
    if req:
        r["required"] = req
    if rec and rec.get("traffic") is not None:
        r["traffic"] = rec["traffic"]
        r["traffic_over_bytes"] = rec["traffic"] / b
        r["traffic_over_model"] = rec["traffic"] / model
        r["hbm_achieved"] = rec["traffic"] / (build_ms / 1e3) / 1e9
        r["hbm_frac"] = r["hbm_achieved"] / HBM_PEAK_GBS
        r["traffic_source"] = "live rocprofv3 --pmc passes of this run (sum over one build's launches)"
        if rec.get("per_kernel"):
            pk = {k: dict(v) for k, v in rec["per_kernel"].items()}
            for k, v in pk.items():
                got = (v.get("read_x2") or 0.0) + (v.get("write") or 0.0)
                v["counted"] = got
                if req and req.get(k):
                    v["required"] = req[k]
                    v["counted_over_required"] = got / req[k]
            r["per_kernel"] = pk
    return r


def reference_side_figure(device, stream, meshes, W, H, cam_rays, eye, orient, mode="kd", pmc=None, child=False,
                          nbuf=1, expect=None):
    """Reference mode on the bench frame: mode "kd" (BM_OPT_REFERENCE_KD) = the reference's kd-tree
    build and first-hit-leaf march on the GPU, every pixel equal to the reference framebuffer;
    mode "hash" (BM_OPT_REFERENCE_HASH) = its alternative hashed uniform grid (Hash.cu).
    child: a counter pass (3 + PMC_STEPS marches, nothing else). nbuf > 1 (kd): also the frames-in-flight
    rate (nbuf render targets on their own streams), each frame checked against the single trace."""
    import torch

    from raytracercuda_amd import beam
    ctx = beam.Context(params=BENCH_PARAMS, device=device, stream=stream.cuda_stream, reference_kd=mode == "kd",
                       reference_hash=mode == "hash")
    sc = beam.IScene.create(ctx)
    keep = beam.upload_meshes(ctx, sc, meshes)
    builds = [sc.updateGPUScene(stats=True)["build_ms"] for _ in range(8)]  # steady state: median of 3rd-8th
    cam = beam.ICamera.create(ctx)
    ctx._check(cam.setInitialRays(W, H, *cam_rays))
    rt = beam.IRenderTarget.createOffscreen(ctx, W, H)
    for _ in range(3):
        ctx._check(cam.trace(eye, orient, sc, rt))
    torch.cuda.synchronize()
    ea, eb = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = (PMC_STEPS if child else 10) if mode == "kd" else 3
    ea.record(stream)
    for _ in range(reps):
        ctx._check(cam.trace(eye, orient, sc, rt))
    eb.record(stream)
    torch.cuda.synchronize()
    ms = ea.elapsed_time(eb) / reps
    kind = rt.traceKind()
    st = sc.kdStats() if mode == "kd" else sc.gridStats()
    ref = rt.read()
    hits = hits_of(ref["packed"])
    inflight = None
    if mode == "kd" and not child and nbuf > 1:
        # frames in flight, as the bench's value: nbuf targets, each on its own HIP stream
        rts = [beam.IRenderTarget.createOffscreen(ctx, W, H) for _ in range(nbuf)]
        streams = [torch.cuda.Stream() for _ in range(nbuf)]
        for r, s_ in zip(rts, streams):
            r.setStream(s_.cuda_stream)
        for i in range(2 * nbuf):
            ctx._check(cam.trace(eye, orient, sc, rts[i % nbuf]))
        ctx.sync()
        torch.cuda.synchronize()
        steps = 10 * nbuf
        t0 = time.perf_counter()
        for i in range(steps):
            ctx._check(cam.trace(eye, orient, sc, rts[i % nbuf]))
        ctx.sync()
        torch.cuda.synchronize()
        per = (time.perf_counter() - t0) / steps * 1e3
        last = rts[(steps - 1) % nbuf].read()
        inflight = {"frames_in_flight": nbuf, "ms_per_frame": per, "mrays_s": W * H / (per / 1e3) / 1e6,
                    "frame_check": all(np.array_equal(last[k], ref[k]) for k in ref)}
        for r in rts:
            r.destroy()
    rt.destroy()
    cam.destroy()
    sc.destroy()
    del keep
    ctx.close()
    out = {"build_ms": float(np.median(builds[2:])), "trace_ms": ms, "mrays_s": W * H / (ms / 1e3) / 1e6,
           "frame_hits": hits, "trace_kind": kind}
    if expect is not None:  # every plane of the expected frame, every pixel
        out["frame_check"] = all(np.array_equal(ref[k].reshape(-1), expect[k].reshape(-1)) for k in expect)
    if inflight:
        out["in_flight"] = inflight
    if mode == "kd":
        out.update({"kd_leaves": int(st[0]), "face_refs": int(st[1])})
        if not child:
            ks = KIND_KERNELS[kind]
            rec, src = pmc_segment(pmc, "reference_mode", "refmode", ks)
            out["roofline"] = roofline(0, ms, ms, rec, src, ks)  # no §8(d) byte model for the kd march: counters only
    else:
        out.update({"cell_face_pairs": int(st[0]), "buckets_used": int(st[1]), "largest_bucket": int(st[2]),
                    "dropped_by_cap": int(st[3])})
    return out


def golden_frame(name, closest_hit):
    """The committed golden frame of a view (tests/golden/views/<name>.npz: the kd oracle's hits, and the
    closest-hit answers at the reference's early-out pixels) as dense packed / tri_id / t planes."""
    with np.load(os.path.join(REPO, "tests", "golden", "views", name + ".npz"), allow_pickle=False) as z:
        rec = {k: z[k] for k in z.files}
    m = json.load(open(os.path.join(REPO, "tests", "golden", "manifest.json")))["views"][name]
    n = m["w"] * m["h"]
    out = {"packed": np.full(n, 0x0000FF00, np.uint32), "tri_id": np.full(n, 0xFFFFFFFF, np.uint32),
           "t": np.full(n, np.inf, np.float32)}
    for pre in ("hit", "div") if closest_hit else ("hit",):
        px = rec[f"{pre}_pixels"]
        out["packed"][px], out["tri_id"][px], out["t"][px] = rec[f"{pre}_packed"], rec[f"{pre}_tri"], rec[f"{pre}_t"]
    return out


def aa_xml_figure(ctx, stream, torch, nbuf):
    """the workload of the reference's only published timing (aa.xml: bmMarchKernel 38.41 ms,
    build 56.5 ms for the f16's two meshes at 500x500 on a GTX 660 Ti; scenes.AA_XML_PUBLISHED): the
    closest-hit BVH4 trace (its frame checked against the golden frame, closest-hit answers at the
    reference's 11 early-out pixels) and reference mode — the reference's kd-tree build and first-hit-leaf
    march, every pixel checked against the golden reference frame."""
    from raytracercuda_amd import scenes
    c = scenes.CONFIGS["aa_xml"]
    wl = Workload(ctx, "aa_xml", torch, stream)
    m = wl.measure(nbuf, SIDE_STEPS, SIDE_WARMUP)
    got = wl.reference_frame()
    want = golden_frame("f16_500", closest_hit=True)
    wl.close()
    rm = reference_side_figure(0, stream, scenes.scene(c["scene"]), c["width"], c["height"], c["rays"], c["eye"],
                               scenes.IDENTITY, nbuf=nbuf, expect=golden_frame("f16_500", closest_hit=False))
    pub = scenes.AA_XML_PUBLISHED
    sf = m["single_frame"]
    return {"scene": "f16 (2 meshes, 4,056 tris)", "width": c["width"], "height": c["height"], "eye": list(c["eye"]),
            "closest_hit": {"build_ms": m["build_ms"], "trace_ms": sf["trace_kernel_ms"],
                            "mrays_s": sf["mrays_s"], "in_flight_mrays_s": m["mrays_s"],
                            "frame_check": bool(all(np.array_equal(got[k].reshape(-1), want[k]) for k in want)),
                            "in_flight_frame_check": m["frame_check"]},
            "reference_mode": {"build_ms": rm["build_ms"], "trace_ms": rm["trace_ms"], "mrays_s": rm["mrays_s"],
                               "frame_check": rm.get("frame_check"),
                               "in_flight_mrays_s": (rm.get("in_flight") or {}).get("mrays_s")},
            "published": pub,
            "speedup_vs_published_march": pub["march_ms"] / rm["trace_ms"],
            "speedup_vs_published_build": pub["build_ms"] / rm["build_ms"]}


# reference mode (the reference's own kd-tree and march) and the hashed grid are measured on C2: the
# bunny of the reference's Content/bunny.zip, the mesh of its golden frames
REFMODE_CONFIG = "c2"
EXTRA_CONFIGS = {"c2": "c2_bunny", "c3": "c3_armadillo_proxy", "c4": "c4_armadillo_4k", "filled": "filled_view",
                 "c5": "c5_merged_proxy_shadow"}


def resolve_config(args, world):
    """--config auto: BASELINE configs[2] (C3) on one GPU, configs[3] (C4) on 2/4/8."""
    if args.config == "auto":
        args.config = "c3" if world == 1 else "c4"
    return args.config


def pmc_child(args, torch, stream):
    """One counter pass (run by tools/pmc.run_live under rocprofv3 --pmc): the bench's workloads, each
    traced PMC_WARMUP + PMC_STEPS times per mode and nothing else non-counting, and the plan of those
    segments written to args.pmc_child for the parent to cut the dispatch list with."""
    from raytracercuda_amd import beam, scenes
    ctx = beam.Context(params=BENCH_PARAMS, device=0, stream=stream.cuda_stream, leaf_size=args.leaf_size, bvh_width=args.bvh_width)
    nbuf = max(1, args.frames_in_flight)
    names = [args.config] + ([] if args.no_extra else [n for n in EXTRA_CONFIGS if n != args.config])
    segs, builds = [], []
    for name in names:
        wl = Workload(ctx, name, torch, stream)
        builds.append([name, 7])
        modes = ([("inflight", nbuf)] if nbuf > 1 else []) + [("single", 1)]
        for mode, nb in modes:
            wl.run(nb, PMC_STEPS, PMC_WARMUP)
            segs.append({"label": f"{name}/{mode}", "kind": wl.kind, "kernels": list(KIND_KERNELS[wl.kind]),
                         "launches": PMC_WARMUP + PMC_STEPS, "warmup": PMC_WARMUP})
        wl.close()
        if name == args.config and not args.no_extra:
            c = scenes.CONFIGS[REFMODE_CONFIG]
            rk = reference_side_figure(0, stream, scenes.scene(c["scene"]), c["width"], c["height"], c["rays"],
                                       c["eye"], scenes.IDENTITY, child=True)["trace_kind"]
            segs.append({"label": "reference_mode", "kind": rk, "kernels": list(KIND_KERNELS[rk]),
                         "launches": 3 + PMC_STEPS, "warmup": 3})
    ctx.close()
    json.dump({"segments": segs, "builds": builds, "stamp": source_stamp()}, open(args.pmc_child, "w"))


def live_counters(args):
    """The counter passes (tools/pmc.py) for this run, before this process touches the GPU."""
    from tools import pmc as tpmc
    child = [a for a in sys.argv[1:]]
    for flag in ("--pmc", "--pmc-keep", "--steps", "--warmup", "--cpu-seconds"):  # drop flag + value
        while flag in child:
            i = child.index(flag)
            del child[i:i + 2]
    child = [a for a in child if not a.startswith(("--pmc=", "--pmc-keep=", "--steps=", "--warmup="))]
    child += ["--no-cpu-baseline"]
    t0 = time.perf_counter()
    summary, note = tpmc.run_live(os.path.join(REPO, "bench.py"), child, keep_dir=args.pmc_keep,
                                  log=lambda m: print(m, file=sys.stderr, flush=True))
    if summary is not None:
        summary["seconds"] = time.perf_counter() - t0
        summary["note"] = note
    return summary, note


def pmc_report(pmc, note):
    """What the counter passes were and whether they all worked (the line's `pmc` field)."""
    from tools import pmc as tpmc
    if pmc is None:
        return {"note": note}
    return {"note": note or "all passes ok", "seconds": pmc.get("seconds"), "errors": pmc.get("errors") or None,
            "groups": [list(g) for g in tpmc.GROUPS], "segments": [x["label"] for x in pmc["plan"]["segments"]],
            "per_launch": "median over each segment's timed launches (warm-up dropped)"}


def single_gpu(args, torch, stream, pmc=None):
    from raytracercuda_amd import beam, scenes
    ctx = beam.Context(params=BENCH_PARAMS, device=0, stream=stream.cuda_stream, leaf_size=args.leaf_size, bvh_width=args.bvh_width)
    wl = Workload(ctx, args.config, torch, stream)
    nbuf = max(1, args.frames_in_flight)
    head = wl.measure(nbuf, args.steps, args.warmup, args.only, pmc=pmc)
    extra = {}
    if not args.no_extra:
        for name, key in EXTRA_CONFIGS.items():
            if name == args.config:
                continue
            w2 = Workload(ctx, name, torch, stream)
            # a fixed, steady-state count whatever --steps is (with 10 steps three frames'
            # fill and drain weighed on the in-flight rate)
            extra[key] = w2.measure(nbuf, SIDE_STEPS, max(args.warmup, SIDE_WARMUP), pmc=pmc)
            w2.close()
        c = scenes.CONFIGS[REFMODE_CONFIG]
        rm = scenes.scene(c["scene"])
        extra["reference_mode"] = reference_side_figure(0, stream, rm, c["width"], c["height"], c["rays"], c["eye"],
                                                        scenes.IDENTITY, pmc=pmc, nbuf=max(1, args.frames_in_flight))
        extra["reference_mode"]["config_id"] = REFMODE_CONFIG
        extra["hashed_grid"] = reference_side_figure(0, stream, rm, c["width"], c["height"], c["rays"], c["eye"],
                                                     scenes.IDENTITY, "hash")
        extra["hashed_grid"]["config_id"] = REFMODE_CONFIG
        extra["aa_xml"] = aa_xml_figure(ctx, stream, torch, max(1, args.frames_in_flight))
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
    ctx, transport, transport_id, fallback = None, None, None, False
    if not shared:
        # the C ABI's own RCCL communicator; every rank must end up on the same transport, so a
        # failure anywhere (no librccl, no unique id, init error) moves all ranks to the
        # torch.distributed gather (multigpu.start_comm: sentinel broadcast + votes)
        def broadcast(obj):
            box = [obj]
            dist.broadcast_object_list(box, src=0)
            return box[0]

        def vote(flag):
            ok = torch.tensor([int(flag)], dtype=torch.int32, device=dev)
            dist.all_reduce(ok, op=dist.ReduceOp.MIN)
            return int(ok[0]) == 1

        ctx, err = multigpu.start_comm(
            rank, beam.comm_unique_id, beam.comm_available,
            lambda: beam.Context(params=BENCH_PARAMS, device=local, stream=stream.cuda_stream, leaf_size=args.leaf_size, planes=planes),
            lambda cx, uid: cx.start_comm(rank, world, uid), broadcast, vote)
        if ctx is not None:
            transport, transport_id = "RCCL send/recv inside libbeam_hip.so (bm_context_start_comm), xGMI", "rccl_lib"
        else:
            torch_gather, fallback = True, True
            transport = f"torch.distributed gather over RCCL (the C-ABI communicator did not start: {err})"
            transport_id = "torch_rccl"
    if torch_gather:
        ctx = beam.Context(params=BENCH_PARAMS, device=local, stream=stream.cuda_stream, leaf_size=args.leaf_size)
        if shared:
            transport = "torch.distributed gather over gloo (shared-device rehearsal: all ranks on one GPU)"
            transport_id = "gloo_shared"
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
    # device-time split of each target's last frame (bm_rt_last_timing): this rank's band trace and
    # the exchange after it; trace = the slowest rank's, gather = rank 0's (it waits for every band)
    split = [-1.0, -1.0]  # none: the torch.distributed gather (rehearsal / fallback) is not timed inside
    if not torch_gather:
        tm = np.array([rt.lastTiming() for rt in rts], np.float64)
        split = [float(tm[:, 0].mean()), float(tm[:, 1].mean())]
    sp = torch.tensor(split, dtype=torch.float64, device="cpu" if shared else dev)
    tmax = sp.clone()
    dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
    out = None
    if rank == 0:
        one = beam.Context(params=BENCH_PARAMS, device=local)  # the same frame traced by this GPU alone
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
        out = {"elapsed": elapsed, "W": W, "H": H, "transport": transport, "transport_id": transport_id,
               "fallback": fallback, "frame_check": bool(check),
               "checked_planes": sorted(got), "build_ms": float(np.median(builds[2:])), "tris": st["num_tris"],
               "frame_hits": hits_of(full["packed"]), "nbuf": nbuf, "scene": c["scene"], "eye": list(eye),
               "frame_bytes": algorithmic_bytes(cnt, W * H, st["bvh_width"]),
               **{k: (float(v) if v >= 0 else None) for k, v in
                  (("trace_ms", tmax[0]), ("gather_ms", sp[1]), ("trace_ms_rank0", sp[0]))}}
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


def multi_record(args, rec, world, common):
    """Rank 0's JSON line at N > 1 from multi_gpu's record (also checked by tests/test_bench_record.py)."""
    rays = rec["W"] * rec["H"]
    step_ms = rec["elapsed"] / args.steps * 1e3
    gathered = "every plane as traced" if args.gather_planes == "all" else (
        "the packed plane" if args.gather_planes == "packed" else "the triangle-id plane (rank 0 reshades)")
    return {**common, "value": rays * args.steps / rec["elapsed"] / 1e6, "ms_per_step": step_ms, "scaling": "strong",
            "config": {"workload": f"{args.config}: {rec['scene']} ({rec['tris']} tris), one fixed {rec['W']}x"
                                   f"{rec['H']} frame, {BAND_H}-row bands round-robin over {world} GPUs, "
                                   f"gather of {gathered} into rank 0 per step: {rec['transport']}; "
                                   f"{rec['nbuf']} frames in flight",
                       "config_id": args.config, "scene": rec["scene"], "tris": rec["tris"],
                       "width": rec["W"], "height": rec["H"], "band_h": BAND_H,
                       "gather_planes": args.gather_planes, "parallelism": f"screen-bands x{world}",
                       # which transport carried the bands, and whether it is the fallback
                       # (the C-ABI communicator failed to start on some rank and every rank moved to
                       # torch.distributed); rccl_lib = the product path
                       "transport": rec["transport_id"], "fallback": bool(rec["fallback"])},
            "trace_ms": rec["trace_ms"], "gather_ms": rec["gather_ms"], "trace_ms_rank0": rec["trace_ms_rank0"],
            "timing_note": "device time of each render target's last frame (HIP events, bm_rt_last_timing), mean "
                           "over the frames-in-flight targets: trace_ms = the slowest rank's band trace, gather_ms = "
                           "rank 0's exchange after its own trace (RCCL receive of every band incl. waiting for the "
                           "slowest rank, scatter, reshade); frames overlap, so they need not add up to ms_per_step",
            "build_ms": rec["build_ms"], "frame_check": rec["frame_check"],
            "checked_planes": rec["checked_planes"], "frame_hits": rec["frame_hits"],
            "gather_bytes_per_frame": rays * (16 if args.gather_planes == "all" else 4) * (world - 1) // world,
            "roofline": compact_roofline(roofline(rec["frame_bytes"] / world, step_ms, step_ms, None,
                                                  "no counter passes at N > 1 (one process per GPU)",
                                                  KIND_KERNELS["cull+quads"], overlapped=True)),
            "roofline_note": "per rank: its share of the frame's algorithmic bytes over the step time (trace + "
                             "gather, frames in flight) under levels.data; no counter passes at N > 1, so the "
                             "HBM fields (traffic, achieved, frac) are null",
            "cpu_baseline": None, "host": platform.node()}


def single_record(args, head, extra, cpu, pmc, pmc_note, common):
    """The full N = 1 record (written to FULL_RECORD): `value` = the configured workload (C3 by default)
    with frames in flight, every side figure with its roofline, limiter and counter details."""
    c = head
    light = bool(head.get("light"))
    return {**common, "value": head["mrays_s"], "ms_per_step": head["ms_per_step"], "scaling": "strong",
            "config": {"workload": f"{args.config}: {c['scene']} ({c['tris']} tris) {c['width']}x"
                                   f"{c['height']} primary rays{' + shadow rays' if light else ''}, "
                                   f"{c['frames_in_flight']} frames in flight (one HIP stream per render "
                                   f"target)",
                       "config_id": args.config, "scene": c["scene"], "tris": c["tris"],
                       "width": c["width"], "height": c["height"], "leaf_size": args.leaf_size,
                       "bvh_width": args.bvh_width, "parallelism": "1 GPU"},
            "build_ms": head["build_ms"], "build_roofline": head["build_roofline"], "trace_kind": head["trace_kind"],
            "trace_kernel_ms": head["trace_kernel_ms"], "frames_in_flight": head["frames_in_flight"],
            "roofline": head["roofline"], "single_frame": head["single_frame"], "per_ray": head["per_ray"],
            "frame_hits": head["frame_hits"], "frame_check": head["frame_check"], "cpu_baseline": cpu,
            **extra, "host": platform.node(),
            "pmc": pmc_report(pmc, pmc_note)}


def _r(x, nd=4):
    """Round for the compact line (floats to nd significant digits; None and ints as they are)."""
    if isinstance(x, float):
        return float(f"{x:.{nd}g}")
    return x


def compact_roofline(r):
    """The contract fields of a roofline plus each level's bytes / achieved / frac and the limiter
    (no raw counters, resources or notes: those stay in the full record)."""
    if not r:
        return r
    out = {k: _r(r.get(k)) for k in ("bound", "achieved", "peak", "unit", "frac", "traffic", "kernel_ms", "step_ms",
                                     "launch_ms")}
    out["kernel"] = r.get("kernel")
    out["launch_overlapped"] = r.get("launch_overlapped")
    lv = {}
    for name, v in (r.get("levels") or {}).items():
        if name == "hbm":  # the contract fields above
            continue
        lv[name] = {k: _r(v.get(k)) for k in ("bytes", "achieved", "peak", "frac")}
    if lv:
        out["levels"] = lv
    lim = r.get("limiter") or {}
    if lim:
        out["limiter"] = {k.replace("wave_time_", ""): _r(v, 3) for k, v in lim.items()}
    return out


def compact_build(b):
    if not b:
        return b
    out = {k: _r(b.get(k)) for k in ("achieved", "peak", "frac", "bytes_per_tri", "traffic", "traffic_over_bytes",
                                      "traffic_over_model", "hbm_frac")}
    out = {k: v for k, v in out.items() if v is not None}
    pk = {k: _r(v.get("counted_over_required"), 3) for k, v in (b.get("per_kernel") or {}).items()
          if v.get("counted_over_required") is not None}
    if pk:
        out["counted_over_required"] = pk
    return out


def compact_side(x):
    """One side figure (another config) in a few numbers."""
    sf = x.get("single_frame") or {}
    rf = x.get("roofline") or {}
    out = {"mrays_s": _r(x.get("mrays_s")), "ms_per_step": _r(x.get("ms_per_step")),
           "trace_kernel_ms": _r(x.get("trace_kernel_ms")), "frame_check": x.get("frame_check"),
           "build_ms": _r(x.get("build_ms")), "single_mrays_s": _r(sf.get("mrays_s")),
           "single_kernel_ms": _r(sf.get("trace_kernel_ms"))}
    for lvl in ("data", "l2", "hbm"):  # each against its own level's peak (data and l2: the L2's)
        f = ((rf.get("levels") or {}).get(lvl) or {}).get("frac")
        if f is not None:
            out[f"{lvl}_frac"] = _r(f, 3)
    if x.get("rays_incl_shadow_per_s_M") is not None:
        out["rays_incl_shadow_per_s_M"] = _r(x["rays_incl_shadow_per_s_M"])
    if x.get("build_roofline", {}).get("traffic_over_bytes") is not None:
        out["build_traffic_over_bytes"] = _r(x["build_roofline"]["traffic_over_bytes"], 3)
    return out


def compact_record(full, full_path=None):
    """The ONE line the driver parses (the 22-25 kB line of round 4 was not parsed): the
    headline, config, roofline, single_frame, build, cpu_baseline and one small dict per side figure;
    the full record is written to `full_path` and named in the line."""
    keep = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data", "config", "source_stamp", "build_ms", "trace_kind", "trace_kernel_ms",
            "frames_in_flight", "frame_hits", "frame_check", "per_ray", "host")
    out = {k: full.get(k) for k in keep if k in full}
    for k in ("value", "ms_per_step", "build_ms", "trace_kernel_ms"):
        if isinstance(out.get(k), float):
            out[k] = _r(out[k], 6)
    out["per_ray"] = {k: _r(v) for k, v in (full.get("per_ray") or {}).items()}
    out["roofline"] = compact_roofline(full.get("roofline"))
    sf = full.get("single_frame")
    if sf:
        out["single_frame"] = {"mrays_s": _r(sf.get("mrays_s")), "ms_per_step": _r(sf.get("ms_per_step")),
                               "trace_kernel_ms": _r(sf.get("trace_kernel_ms")), "trace_kind": sf.get("trace_kind"),
                               "roofline": compact_roofline(sf.get("roofline"))}
    out["build_roofline"] = compact_build(full.get("build_roofline"))
    cpu = full.get("cpu_baseline")
    if cpu:
        out["cpu_baseline"] = {k: _r(cpu.get(k)) for k in ("value", "unit", "cores", "kind", "algorithm",
                                                            "single_thread_mrays_s", "build_ms", "cpu_model")}
        out["cpu_baseline"]["sample"] = cpu.get("sample")
        if cpu.get("lbvh_port"):
            out["cpu_baseline"]["lbvh_port_mrays_s"] = _r(cpu["lbvh_port"].get("mrays_s"))
    else:
        out["cpu_baseline"] = cpu
    side = {}
    for key in EXTRA_CONFIGS.values():
        if key in full:
            side[key] = compact_side(full[key])
    if side:
        out["side"] = side
    rm = full.get("reference_mode")
    if rm:
        out["reference_mode"] = {"config_id": rm.get("config_id"), "build_ms": _r(rm.get("build_ms")),
                                 "trace_ms": _r(rm.get("trace_ms")), "mrays_s": _r(rm.get("mrays_s")),
                                 "in_flight_mrays_s": _r((rm.get("in_flight") or {}).get("mrays_s")),
                                 "frame_check": (rm.get("in_flight") or {}).get("frame_check"),
                                 "hbm_frac": _r((((rm.get("roofline") or {}).get("levels") or {}).get("hbm") or {})
                                                .get("frac"), 3)}
    aa = full.get("aa_xml")
    if aa:
        out["side"] = dict(out.get("side") or {}, aa_xml={
            "closest_hit": {k: _r(v) for k, v in aa["closest_hit"].items()},
            "reference_mode": {k: _r(v) for k, v in aa["reference_mode"].items()},
            "published_march_ms": aa["published"]["march_ms"], "published_build_ms": _r(aa["published"]["build_ms"]),
            "speedup_vs_published_march": _r(aa["speedup_vs_published_march"]),
            "speedup_vs_published_build": _r(aa["speedup_vs_published_build"])})
    hg = full.get("hashed_grid")
    if hg:
        out["hashed_grid"] = {k: _r(hg.get(k)) for k in ("config_id", "build_ms", "trace_ms", "mrays_s", "frame_hits",
                                                           "dropped_by_cap")}
    p = full.get("pmc") or {}
    out["pmc"] = {"note": p.get("note"), "seconds": _r(p.get("seconds"), 3), "errors": p.get("errors")}
    if full_path:
        out["full_record"] = full_path
    return out


def write_full(full):
    """Write the full record next to the run's outputs; returns the path named in the line (or None)."""
    path = os.path.join(REPO, FULL_RECORD)
    try:
        os.makedirs(os.path.dirname(path), exist_ok=True)
        with open(path, "w") as f:
            json.dump(full, f, indent=1)
        return FULL_RECORD
    except OSError as e:
        print(f"warning: full record not written: {e}", file=sys.stderr)
        return None


def finite(x):
    """The record with every non-finite float replaced by None (strict JSON for the driver)."""
    if isinstance(x, float):
        return x if np.isfinite(x) else None
    if isinstance(x, dict):
        return {k: finite(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return [finite(v) for v in x]
    return x


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def self_launch(args, argv):
    """`bench.py --gpus N` (N > 1) started without a launcher: run N ranks as a CHILD torch.distributed.run
    (one process per GPU, 127.0.0.1 rendezvous), before this process touches the GPU; relay the ranks'
    output, check that exactly one JSON line came back with n_gpus == N and print it. Returns the exit
    code (non-zero when the ranks failed or the line is missing: never a mislabelled 1-GPU line)."""
    import subprocess
    n = args.gpus
    dry = os.environ.get("BM_BENCH_DRY_RUN") == "1"
    shared = os.environ.get("BM_BENCH_SHARED_DEVICE") == "1"
    if not dry and not shared:
        import torch  # device_count() does not initialise the GPU on this image
        have = torch.cuda.device_count()
        if have < n:
            print(f"bench.py: --gpus {n} but only {have} GPU(s) visible; no line printed", file=sys.stderr)
            return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.abspath(__file__), *argv]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS=os.environ.get("OMP_NUM_THREADS", "1"))
    print(f"bench.py: launching {n} ranks: {' '.join(cmd)}", file=sys.stderr, flush=True)
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True, env=env, cwd=REPO)
    lines = []
    for ln in p.stdout:  # streamed: progress stays visible; stdout carries only the JSON line
        if ln.startswith("{"):
            try:
                lines.append(json.loads(ln))
                continue
            except ValueError:
                pass
        sys.stderr.write(ln)
        sys.stderr.flush()
    rc = p.wait()
    good = [x for x in lines if x.get("n_gpus") == n]
    if rc != 0 or len(lines) != 1 or len(good) != 1:
        print(f"bench.py: the {n}-rank run exited {rc} with {len(lines)} JSON line(s) "
              f"({len(good)} with n_gpus == {n}); no line printed", file=sys.stderr)
        return rc or 3
    print(json.dumps(good[0], allow_nan=False), flush=True)
    return 0


def dry_run(args, world, rank):
    """BM_BENCH_DRY_RUN=1 (CPU tests of the launcher): no GPU; the ranks meet over gloo and rank 0 prints a
    stub line with the number of ranks that reported in."""
    import torch
    import torch.distributed as dist
    seen = world
    if world > 1:
        dist.init_process_group("gloo")
        t = torch.ones(1)
        dist.all_reduce(t)
        seen = int(t[0])
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": 0.0, "unit": "Mrays/s", "n_gpus": world, "steps": args.steps,
                          "warmup": args.warmup, "dry_run": True, "ranks_seen": seen}), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ and not args.pmc_child:
        sys.exit(self_launch(args, sys.argv[1:]))
    if world != args.gpus:
        # a launcher with another rank count: measuring would print a line for the wrong N
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; no line printed", file=sys.stderr)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    if os.environ.get("BM_BENCH_DRY_RUN") == "1":
        dry_run(args, world, rank)
        return
    import torch
    import torch.distributed as dist

    resolve_config(args, world)
    if args.pmc_child:  # one counter pass under rocprofv3 (tools/pmc.py)
        torch.cuda.set_device(0)
        pmc_child(args, torch, torch.cuda.current_stream())
        return
    pmc, pmc_note = None, "off"
    if world == 1 and (args.pmc == "on" or (args.pmc == "auto" and args.only == "both")):
        from tools import pmc as tpmc
        if tpmc.under_profiler():
            pmc_note = "skipped: already running under a profiler"
        else:  # before this process touches the GPU: the passes are child processes
            pmc, pmc_note = live_counters(args)
    local = int(os.environ.get("LOCAL_RANK", "0"))
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
        head, extra, cpu = single_gpu(args, torch, stream, pmc)
        full = finite(single_record(args, head, extra, cpu, pmc, pmc_note, common))
        print(json.dumps(compact_record(full, write_full(full)), allow_nan=False), flush=True)
        return
    rec = multi_gpu(args, torch, dist, rank, world, local, shared)
    if rank == 0:
        print(json.dumps(finite(multi_record(args, rec, world, common)), allow_nan=False), flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
