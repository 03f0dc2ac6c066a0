"""Decompositions of the frame sequence across ranks (one process per GPU).

Frames (the default, weak scaling): frames are independent units of work,
so rank r renders whole frames r, r+N, r+2N, ... of the one-GPU sequence;
no data crosses ranks.

Row bands (strong scaling, one frame split):
The frame is cut into bands of B rows dealt round-robin to the ranks
("interleaved row bands"): the scene sits in the middle of the reference
camera's view, so contiguous row blocks would leave the outer ranks idle.
Every rank renders its rows with the GLOBAL pixel index (RNG subsequence and
jitter), so the gathered frame is byte-identical to a one-GPU render.
"""
from __future__ import annotations

import numpy as np

from ._lib import Rows


def rows_of_rank(h: int, band: int, rank: int, world: int) -> np.ndarray:
    y = np.arange(h)
    return y[(y // band) % world == rank]


def band_rows(h: int, band: int, rank: int, world: int) -> Rows:
    """bih_rows for rank `rank`: local row r -> y = rank*band + (r//band)*band*world + r%band."""
    n = int(rows_of_rank(h, band, rank, world).size)
    return Rows(rank * band, n, band, world)


def max_rows(h: int, band: int, world: int) -> int:
    return max(int(rows_of_rank(h, band, r, world).size) for r in range(world))


def assemble(parts, h: int, band: int, world: int) -> np.ndarray:
    """Inverse of the tiling: parts[r] holds rank r's rows (padded rows ignored)."""
    w = parts[0].shape[1]
    out = np.zeros((h, w), parts[0].dtype)
    for r in range(world):
        ys = rows_of_rank(h, band, r, world)
        out[ys] = parts[r][: ys.size]
    return out


def gather_order(h: int, band: int, world: int) -> np.ndarray:
    """Row index into the all-gathered [world * max_rows, W] buffer (rank r's
    rows at r * max_rows) for every frame row y: frame = gathered[order]."""
    mrows = max_rows(h, band, world)
    order = np.empty(h, np.int64)
    for r in range(world):
        ys = rows_of_rank(h, band, r, world)
        order[ys] = np.arange(ys.size) + r * mrows
    return order


class BandGather:
    """The exchange step of the row-band decomposition: every rank's bands go
    to the root with ONE gather per frame (torch.distributed ``gather``; on
    the nccl backend that is RCCL ncclSend/ncclRecv to the root over xGMI,
    the pattern of ncclGather, rccl.h:745) and the root lays them out in
    frame order with one device permutation.  Non-root ranks receive nothing
    (an all-gather would send every rank the whole frame).

    One instance per frame in flight: it owns that frame's receive buffer.
    ``local`` is this rank's render output, rows in local order (at least
    max_rows * w elements; rows past the rank's own are padding and ignored);
    ``frame`` (root only) receives the h x w frame."""

    def __init__(self, dist, h: int, w: int, band: int, rank: int, world: int, device,
                 root: int = 0):
        import torch
        self.dist, self.h, self.w, self.rank, self.world, self.root = dist, h, w, rank, world, root
        self.mrows = max_rows(h, band, world)
        n = self.mrows * w
        self.recv = None
        self.parts = None
        self.order = None
        if rank == root:
            self.recv = torch.empty(world * n, dtype=torch.int32, device=device)
            self.parts = [self.recv[r * n:(r + 1) * n] for r in range(world)]
            self.order = torch.from_numpy(gather_order(h, band, world)).to(device)

    def __call__(self, local, frame=None):
        import torch
        send = local[: self.mrows * self.w]
        if self.rank == self.root:
            self.dist.gather(send, self.parts, dst=self.root)
            if frame is not None:
                torch.index_select(self.recv.view(self.world * self.mrows, self.w), 0, self.order,
                                   out=frame.view(self.h, self.w))
        else:
            self.dist.gather(send, None, dst=self.root)


def frame_of_step(base: int, k: int, rank: int, world: int) -> int:
    """Frame index rank `rank` renders at its k-th step when whole frames are
    dealt round-robin: steps k of all ranks cover frames base + kN .. base + kN + N-1."""
    return base + k * world + rank
