"""Multi-rank screen-band partition + single gather, world_size 2/3 over gloo on CPU.

Each rank fills its band buffer int32[3, rows, W] (packed, tri id, t bits) for exactly the global
rows raytracercuda_amd.multigpu.local_to_global_rows assigns it (here with the CPU oracle as the
per-pixel tracer, test-only; on the GPU box the same buffer is written by the HIP kernel through
bm_camera_trace_bands), the buffers meet on rank 0 through multigpu.gather_to_root, and
multigpu.reassemble_torch must reproduce the single-process frame bit-exactly.
"""
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
