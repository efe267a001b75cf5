"""CPU, multi-process (gloo, world size 2, 3 and 8 -- the 8-GPU config's rank count): the N>1 frame
path of bench.py — round-robin 8x8 tile shards, per-rank packed buffers, FrameGather's gather to rank 0, and reassembly — gives the
exact single-process frame.  Rendering here is the CPU oracle (the GPU is not available); the
GPU-side tests check gi_render_device's packed output and gi_unshard_device against the same
layout (test_gpu_parity.py::test_sharded_render_equals_single, test_unshard_matches_host_layout)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle_util as U


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, w, h, scn, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from importlib import import_module
        S = import_module("2019global_amd.shard")
        full = U.oracle_render(scn, w, h, threads=1)["rgb"].reshape(-1, 3)
        fg = S.FrameGather(torch, dist, w, h, world, rank, "cpu")
        pp = S.packed_pixels(w, h, world, rank)
        mine = np.zeros((len(pp), 3))
        mine[pp >= 0] = full[pp[pp >= 0]]      # "render" this rank's tiles
        fg.buf.copy_(torch.from_numpy(mine.reshape(-1)))
        fg.buf8.zero_()
        fg.gather()
        if rank == 0:
            allp = fg.packed_all.numpy().reshape(-1, 3)
            frame = allp[S.unshard_index(w, h, world)]
            q.put(bool(U.bits_equal(frame, full).all()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 8])
def test_sharded_gather_reassembles_frame(world):
    S = U.scenes()
    w, h = 61, 43   # ragged: partial tiles on both edges
    scn = S.cornell_scene().to_scn()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, w, h, scn, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(180)
        assert p.exitcode == 0
    assert q.get(timeout=10) is True


def test_layout_covers_every_pixel_once():
    from importlib import import_module
    S = import_module("2019global_amd.shard")
    for w, h, n in [(61, 43, 2), (64, 64, 8), (1920, 1080, 8), (17, 5, 3)]:
        seen = np.concatenate([S.packed_pixels(w, h, n, r) for r in range(n)])
        seen = seen[seen >= 0]
        assert len(seen) == w * h and len(np.unique(seen)) == w * h
        assert S.tiles_per_rank(w, h, n) == U.pkg().shard_tiles(w, h, n)
