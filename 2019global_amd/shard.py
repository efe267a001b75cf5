"""Tile sharding of one frame over N ranks (one process per GPU) and the gather to rank 0.

Layout (include/gi.h, GI_TILE): the frame is cut into 8x8-pixel tiles in row-major tile order;
tile t belongs to rank t % N (round-robin, so the ~100x per-ray cost variance between scene
centre and background spreads evenly).  Rank r renders its tiles into a packed
buffer [n_local][64][3] (n_local = ceil(T / N), padded so every rank's buffer has the same size)
with gi_render_device; rank 0 gathers the N buffers (one ncclGather = torch.distributed.gather on
the nccl backend, RCCL over xGMI: N-1 point-to-point streams into rank 0) and reassembles the
frame with gi_unshard_device.  The index maps below are the host-side statement of that layout
(used by tests and for checks); the product reassembly runs on the GPU.
"""
from __future__ import annotations

import numpy as np

TILE = 8


def n_tiles(w: int, h: int) -> int:
    return ((w + TILE - 1) // TILE) * ((h + TILE - 1) // TILE)


def tiles_per_rank(w: int, h: int, n: int) -> int:
    return -(-n_tiles(w, h) // n)


def packed_pixels(w: int, h: int, n: int, rank: int) -> np.ndarray:
    """Frame pixel index (y*w + x) of every slot of rank's packed buffer; -1 for padding slots."""
    tx = (w + TILE - 1) // TILE
    T = n_tiles(w, h)
    nl = tiles_per_rank(w, h, n)
    lt = np.arange(nl)[:, None]
    lane = np.arange(TILE * TILE)[None, :]
    t = rank + lt * n
    x = (t % tx) * TILE + (lane & 7)
    y = (t // tx) * TILE + (lane >> 3)
    ok = (t < T) & (x < w) & (y < h)
    return np.where(ok, y * w + x, -1).reshape(-1)


def unshard_index(w: int, h: int, n: int) -> np.ndarray:
    """For each frame pixel, its slot in the rank-concatenated packed buffers."""
    per = tiles_per_rank(w, h, n) * TILE * TILE
    out = np.full(w * h, -1, np.int64)
    for r in range(n):
        pp = packed_pixels(w, h, n, r)
        sel = pp >= 0
        out[pp[sel]] = r * per + np.nonzero(sel)[0]
    assert (out >= 0).all()
    return out


class FrameGather:
    """Per-rank buffers for one sharded frame and the gather to rank 0 (torch.distributed).

    `render(buf, buf8)` fills this rank's packed buffers (the caller's renderer: gi_render_device
    on the GPU); `gather()` collects them on rank 0 into `packed_all` / `packed_all8`, which
    gi_unshard_device (or `unshard_index` on the host) turns into the frame."""

    def __init__(self, torch, dist, w: int, h: int, world: int, rank: int, device):
        self.torch, self.dist = torch, dist
        self.w, self.h, self.world, self.rank = w, h, world, rank
        self.per = tiles_per_rank(w, h, world) * TILE * TILE * 3
        self.buf = torch.empty(self.per, dtype=torch.float64, device=device)
        self.buf8 = torch.empty(self.per, dtype=torch.uint8, device=device)
        if rank == 0:
            self.packed_all = torch.empty(world * self.per, dtype=torch.float64, device=device)
            self.packed_all8 = torch.empty(world * self.per, dtype=torch.uint8, device=device)
            # views into the concatenated buffer: gather writes each rank's part in place
            self.parts = list(self.packed_all.split(self.per))
            self.parts8 = list(self.packed_all8.split(self.per))
        else:
            self.packed_all = self.packed_all8 = self.parts = self.parts8 = None

    def gather(self, radiance: bool = True) -> None:
        """Gathers the RGB888 frame (the reference's Image, image.h:14-16) and, unless
        radiance=False, the fp64 radiance as well (8x the bytes: diagnostics / parity)."""
        pairs = [(self.buf8, self.parts8)] + ([(self.buf, self.parts)] if radiance else [])
        if self.dist.get_backend() == "gloo" and self.buf.is_cuda:
            # gloo gathers host tensors only (rehearsal path: several ranks sharing one device)
            for src, dst in pairs:
                host = [p.cpu() for p in dst] if self.rank == 0 else None
                self.dist.gather(src.cpu(), host, dst=0)
                if self.rank == 0:
                    for d, s in zip(dst, host):
                        d.copy_(s)
            return
        for src, dst in pairs:
            self.dist.gather(src, dst, dst=0)
