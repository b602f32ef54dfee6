"""Multi-rank screen-band partition + single gather, world_size 2/3 over gloo on CPU.

Each rank fills its band buffer int32[3, rows, W] (packed, tri id, t bits) for exactly the global
rows raytracercuda_amd.multigpu.local_to_global_rows assigns it (here with the CPU oracle as the
per-pixel tracer, test-only; on the GPU box the same buffer is written by the HIP kernel through
bm_camera_trace_bands), the buffers meet on rank 0 through multigpu.gather_to_root, and
multigpu.reassemble_torch must reproduce the single-process frame bit-exactly.
"""
import datetime
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from raytracercuda_amd import multigpu, scenes

W, H, BAND = 48, 70, 16


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _frame_planes(packed, tri, t):
    return np.stack([packed.view(np.int32), tri.view(np.int32), t.view(np.int32)])


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import Oracle
        o = Oracle()
        err, rays = o.camera_rays(W, H, *scenes.RAYS_1080)
        bvh = o.bvh_build(scenes.load_mesh("bunny"), 4)
        packed, tri, t = bvh.render(rays, scenes.BUNNY_EYE, scenes.IDENTITY)
        full = _frame_planes(packed, tri, t).reshape(3, H, W)
        rows = multigpu.local_to_global_rows(H, BAND, world, rank)
        buf = torch.zeros((3, rows.size, W), dtype=torch.int32)
        for lr, g in enumerate(rows):
            if g >= 0:  # this rank traces global row g into local row lr
                buf[:, lr] = torch.from_numpy(full[:, g].copy())
        gathered = torch.empty((world, 3, rows.size, W), dtype=torch.int32) if rank == 0 else None
        multigpu.gather_to_root(buf, rank, world, gathered)
        if rank == 0:
            frame = multigpu.reassemble_torch(gathered, H, BAND)
            q.put(bool(torch.equal(frame, torch.from_numpy(full))))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_band_gather_reassembles_frame(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert q.get(timeout=5) is True


def test_band_layout_properties():
    for h, bh, world in [(1080, 16, 1), (1080, 16, 8), (70, 16, 3), (2160 * 2, 16, 8), (5, 16, 4)]:
        seen = []
        for r in range(world):
            rows = multigpu.local_to_global_rows(h, bh, world, r)
            assert rows.size == multigpu.rows_per_rank(h, bh, world)
            seen.extend(rows[rows >= 0].tolist())
        assert sorted(seen) == list(range(h))  # every row exactly once, over all ranks
        parts = np.stack([np.where(multigpu.local_to_global_rows(h, bh, world, r) >= 0,
                                   multigpu.local_to_global_rows(h, bh, world, r), -7)[None, :, None]
                          for r in range(world)])
        frame = multigpu.reassemble_np(parts, h, bh)
        assert np.array_equal(frame[0, :, 0], np.arange(h))


class _Ctx:
    def __init__(self, rank, log):
        self.rank, self.log = rank, log

    def close(self):
        self.log.append(f"closed {self.rank}")


def _comm_worker(rank, world, port, q, fail):
    """multigpu.start_comm over gloo with stand-ins for the C ABI calls; `fail` picks what breaks.
    join() stands in for bm_context_start_comm: like ncclCommInitRank it is a collective (a gloo
    barrier under a timeout), so a rank entering it alone blocks — the test fails with a timeout
    instead of passing if start_comm ever lets some ranks into the collective without the others."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        log = []

        def unique_id():
            if fail == "unique_id":
                raise RuntimeError("no librccl")
            return b"x" * 128

        def probe():
            if fail == "probe" and rank == world - 1:
                raise RuntimeError("librccl.so.1 not found")

        def make_ctx():
            if fail == "context" and rank == 1:  # the device setup fails on one rank (stream, memory)
                raise RuntimeError("hipStreamCreate failed")
            return _Ctx(rank, log)

        def join(ctx, uid):
            assert uid == b"x" * 128 and isinstance(ctx, _Ctx)
            log.append(f"joined {rank}")
            dist.monitored_barrier(timeout=datetime.timedelta(seconds=20))  # the collective
            if fail == "join" and rank == 2:  # a failure reported after the collective
                raise RuntimeError("ncclCommInitRank: internal error")

        def broadcast(obj):
            box = [obj]
            dist.broadcast_object_list(box, src=0)
            return box[0]

        def vote(flag):
            t = torch.tensor([int(flag)], dtype=torch.int32)
            dist.all_reduce(t, op=dist.ReduceOp.MIN)
            return int(t[0]) == 1

        ctx, err = multigpu.start_comm(rank, unique_id, probe, make_ctx, join, broadcast, vote)
        dist.barrier()  # every rank left start_comm: no collective is left waiting
        q.put((rank, ctx is not None, bool(err), log))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("fail", [None, "unique_id", "probe", "context", "join"])
def test_start_comm_all_ranks_take_one_transport(fail):
    """The N > 1 bench path's transport choice: whatever fails on whichever rank,
    every rank leaves start_comm (no rank waits alone in the collective) and all of them either keep
    the RCCL context or fall back; a context that was created is closed when another rank failed."""
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_comm_worker, args=(r, world, port, q, fail)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    res = sorted(q.get(timeout=5) for _ in range(world))
    assert {r[1] for r in res} == {fail is None}  # one transport on every rank
    if fail is not None:
        assert all(r[2] for r in res if r[0] == 0 or fail not in ("context", "join"))  # the reason travels
    if fail == "context":  # ranks 0 and 2 created their context, nobody entered the collective
        assert res[0][3] == ["closed 0"] and res[2][3] == ["closed 2"] and res[1][3] == []
    if fail == "join":  # all entered the collective together, then all closed
        assert all(r[3] == [f"joined {r[0]}", f"closed {r[0]}"] for r in res)
    if fail is None:
        assert all(r[3] == [f"joined {r[0]}"] for r in res)
