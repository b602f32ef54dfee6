"""Screen-band partition of a frame over the GPUs of one node + one RCCL gather.

The reference is single-GPU (Program.cpp:122-124). Primary rays are independent, so the frame is
cut into horizontal bands of `band_h` rows dealt round-robin to the ranks (band b -> rank b % N,
which balances the load better than contiguous row blocks when the subject sits mid-frame). Every
rank builds the same BVH from the same meshes (the build is deterministic, so replicas are
bit-identical and need no broadcast), traces its bands into a compact local buffer, and the buffers
travel to rank 0 in a single gather over RCCL/xGMI (torch.distributed "nccl" backend); rank 0 puts
the bands back in frame order. One process per GPU; launched by torch.distributed.run.

Per-rank buffer: int32[3, rows, W] = (packed u32, triangle id u32, t f32 bits): 12 B / pixel.
"""
from __future__ import annotations

import numpy as np


def num_bands(height: int, band_h: int) -> int:
    return (height + band_h - 1) // band_h


def rows_per_rank(height: int, band_h: int, world: int) -> int:
    """Rows of every rank's (equal-size, padded) local buffer."""
    return ((num_bands(height, band_h) + world - 1) // world) * band_h


def local_to_global_rows(height: int, band_h: int, world: int, rank: int) -> np.ndarray:
    """Global frame row of each local row of `rank`'s buffer (-1 for padding rows). The trace
    kernel applies the same map (bm_camera_trace_bands: band_step = world, band_first = rank)."""
    lr = np.arange(rows_per_rank(height, band_h, world))
    g = ((lr // band_h) * world + rank) * band_h + lr % band_h
    return np.where(g < height, g, -1)


def gather_to_root(buf, rank: int, world: int, gathered=None, async_op: bool = False):
    """The single exchange step: every rank's band buffer into rank 0 (torch.distributed gather;
    RCCL over xGMI with the "nccl" backend, gloo on CPU). `gathered` is [world, *buf.shape] on rank 0.
    async_op: return the collective's work handle (RCCL runs on its own stream) instead of waiting."""
    import torch
    import torch.distributed as dist
    if world == 1:
        if gathered is not None:
            gathered[0].copy_(buf)
        return None
    if buf.is_cuda and dist.get_backend() == "gloo":  # rehearsal on one device: stage through host
        host = buf.cpu()
        if rank == 0:
            parts = [host.clone() for _ in range(world)]
            dist.gather(host, gather_list=parts, dst=0)
            gathered.copy_(torch.stack(parts))
        else:
            dist.gather(host, dst=0)
        return None
    if rank == 0:
        return dist.gather(buf, gather_list=list(gathered.unbind(0)), dst=0, async_op=async_op)
    return dist.gather(buf, dst=0, async_op=async_op)


def reassemble_np(parts: np.ndarray, height: int, band_h: int) -> np.ndarray:
    """parts[N, P, rows, W] (rank-major) -> frame[P, height, W]; band b came from rank b % N."""
    n, p, rows, w = parts.shape
    nbl = rows // band_h
    x = parts.reshape(n, p, nbl, band_h, w).transpose(1, 2, 0, 3, 4)
    return x.reshape(p, nbl * n * band_h, w)[:, :height]


def reassemble_torch(parts, height: int, band_h: int):
    """Same as reassemble_np for a torch tensor [N, P, rows, W] (one device copy kernel)."""
    n, p, rows, w = parts.shape
    nbl = rows // band_h
    x = parts.reshape(n, p, nbl, band_h, w).permute(1, 2, 0, 3, 4)
    return x.reshape(p, nbl * n * band_h, w)[:, :height]


def start_comm(rank: int, make_unique_id, probe, make_ctx, join, broadcast, vote):
    """Start the C ABI's RCCL communicator on every rank, or on none (bench.py --gpus N).

    Every rank must end on the same transport, and the communicator start (ncclCommInitRank) is a
    collective that waits for all ranks, so no rank may enter it unless every rank can: rank 0 makes
    the unique id (a None sentinel travels instead when that fails, so the broadcast still completes
    on every rank); every rank probes that RCCL resolves (probe()) and creates its plain device
    context (make_ctx(): stream, device memory, hipSetDevice — the steps that can fail locally); one
    vote (vote(flag) -> the minimum over ranks) decides whether anyone enters join(ctx, uid) (the
    collective, bm_context_start_comm); a second vote after it decides whether the communicators are
    kept. A failure inside the collective itself is RCCL's to report on every rank.
    broadcast(obj) returns rank 0's obj on every rank. Returns (ctx or None, error text)."""
    err, uid = "", None
    if rank == 0:
        try:
            uid = make_unique_id()
        except Exception as e:  # noqa: BLE001 - reported to the caller, never hidden
            err = f"rank 0 could not make an RCCL unique id: {e}"
    uid = broadcast(uid)
    ctx = None
    if uid is not None:
        try:
            probe()
            ctx = make_ctx()
        except Exception as e:  # noqa: BLE001
            err = f"rank {rank}: {e}"
    if not vote(0 if ctx is None else 1):
        if ctx is not None:
            ctx.close()
        return None, err or "RCCL or the device context unavailable on another rank"
    joined = False
    try:
        join(ctx, uid)
        joined = True
    except Exception as e:  # noqa: BLE001
        err = f"rank {rank}: {e}"
    if not vote(1 if joined else 0):
        ctx.close()
        return None, err or "the communicator failed to start on another rank"
    return ctx, ""


class BandRenderer:
    """One rank's share of a band-partitioned frame (GPU path: libbeam_hip.so + torch.distributed).

    ctx must enqueue on torch's current stream (Context(stream=torch.cuda.current_stream().cuda_stream))
    so the trace and the collectives are ordered against it.

    planes: "packed" gathers the reference's framebuffer (0x00RRGGBB, 4 B/pixel, Beam.h's render
    target); "full" also gathers triangle ids and t (12 B/pixel). Every rank keeps all three planes
    of its own bands either way.
    Pipelining: `frames_in_flight` band buffers (at least two when N > 1) alternate, each a render
    target on its own HIP stream (bm_rt_set_stream), so the trace of frame k+1 starts while frame
    k's trace drains (its workgroups take the CUs frame k's tail leaves idle) and the gather of frame
    k (RCCL, ordered after the trace on that buffer's stream) overlaps the traces after it; a buffer
    is traced into again only after its previous gather finished.
    """

    def __init__(self, ctx, scene, camera, width: int, height: int, band_h: int, rank: int, world: int,
                 device, planes: str = "packed", frames_in_flight: int = 3):
        import torch

        from .beam import IRenderTarget

        self.torch = torch
        self.ctx, self.scene, self.cam = ctx, scene, camera
        self.width, self.height, self.band_h = width, height, band_h
        self.rank, self.world = rank, world
        self.nplanes = 1 if planes == "packed" else 3
        self.rows = rows_per_rank(height, band_h, world)
        nbuf = max(1, frames_in_flight, 2 if world > 1 else 1)
        self.nbuf = nbuf
        self.bufs = [torch.zeros((3, self.rows, width), dtype=torch.int32, device=device) for _ in range(nbuf)]
        self.rts = [IRenderTarget.createExternal(ctx, width, self.rows, width * 4, b[0].data_ptr(),
                                                 b[1].data_ptr(), b[2].data_ptr(), 0, keepalive=b)
                    for b in self.bufs]
        # one stream per buffer when frames overlap; else everything on the context stream
        self.streams = [torch.cuda.Stream(device=device) for _ in range(nbuf)] if nbuf > 1 else [None]
        for rt, st in zip(self.rts, self.streams):
            if st is not None:
                rt.setStream(st.cuda_stream)
        self.gathered = ([torch.empty((world, self.nplanes, self.rows, width), dtype=torch.int32, device=device)
                          for _ in range(nbuf)] if rank == 0 else None)
        self.pending = [None] * nbuf
        self.consumed = [False] * nbuf  # frame() handed the slot's frame out: order its reuse after the reader
        self.i = 0
        self.last = 0

    @property
    def buf(self):
        return self.bufs[self.last]

    @property
    def rt(self):
        return self.rts[self.i % len(self.bufs)]

    def stream(self):
        """The torch stream the next trace runs on (torch's current stream without frames in flight)."""
        st = self.streams[self.i % len(self.bufs)]
        return st if st is not None else self.torch.cuda.current_stream()

    def acquire(self):
        """Order the next trace after the gather still reading its buffer and after the consumer of
        its last frame: everything enqueued on the caller's current stream up to now, which includes
        the reads the caller issued after frame() (stream waits, no host block)."""
        slot = self.i % len(self.bufs)
        if self.pending[slot] is not None:
            with self.torch.cuda.stream(self.stream()):
                self.pending[slot].wait()
            self.pending[slot] = None
        if self.consumed[slot]:
            cur = self.torch.cuda.current_stream()
            if self.stream() != cur:
                self.stream().wait_stream(cur)
            self.consumed[slot] = False

    def trace(self, eye, orient, light=None) -> int:
        """This rank's bands; with a light also their shadow rays (the shadow plane stays local: the
        gather carries the int32 planes only)."""
        self.acquire()
        slot = self.i % len(self.bufs)
        if light is not None:
            return self.cam.traceShadowBands(eye, orient, self.scene, self.rts[slot], self.band_h, self.world,
                                             self.rank, light)
        return self.cam.traceBands(eye, orient, self.scene, self.rts[slot], self.band_h, self.world, self.rank)

    def gather(self):
        """Single gather of every rank's band buffer into rank 0 (RCCL over xGMI), asynchronous."""
        slot = self.i % len(self.bufs)
        if self.world > 1:
            dst = self.gathered[slot] if self.rank == 0 else None
            with self.torch.cuda.stream(self.stream()):  # RCCL orders itself after this buffer's trace
                self.pending[slot] = gather_to_root(self.bufs[slot][: self.nplanes], self.rank, self.world, dst,
                                                    async_op=True)
        self.last = slot
        self.i += 1

    def frame(self):
        """Rank 0: the last gathered frame, int32[planes, H, W] (packed[, tri id, t bits]) on the device.
        The slot is traced into again only after the work the caller enqueued on its current stream
        before that trace (acquire() orders the slot's stream after it)."""
        cur = self.torch.cuda.current_stream()
        if self.world == 1:
            if self.streams[self.last] is not None:
                cur.wait_stream(self.streams[self.last])
            out = self.bufs[self.last][:, : self.height]
        else:
            assert self.rank == 0
            if self.pending[self.last] is not None:
                self.pending[self.last].wait()
                self.pending[self.last] = None
            out = reassemble_torch(self.gathered[self.last], self.height, self.band_h)
        self.consumed[self.last] = True
        return out

    def close(self):
        for w in self.pending:
            if w is not None:
                w.wait()
        for rt in self.rts:
            rt.destroy()
