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


def gather_order(h: int, band: int, world: int, frames: int = 1) -> np.ndarray:
    """Row index into the gathered [world * frames * max_rows, W] buffer (rank
    r's rows of frame f at (r * frames + f) * max_rows) for every row y of
    every frame f: frames = gathered[order].view(frames, h, W)."""
    mrows = max_rows(h, band, world)
    order = np.empty(frames * h, np.int64)
    for f in range(frames):
        for r in range(world):
            ys = rows_of_rank(h, band, r, world)
            order[f * h + ys] = np.arange(ys.size) + (r * frames + f) * mrows
    return order


class BandGather:
    """The exchange step of the row-band decomposition: every rank's bands go
    to the root with ONE gather per frame (torch.distributed ``gather``; on
    the nccl backend that is RCCL ncclSend/ncclRecv to the root over xGMI,
    the pattern of ncclGather, rccl.h:745) and the root lays them out in
    frame order with one device permutation.  Non-root ranks receive nothing
    (an all-gather would send every rank the whole frame).

    One instance per group of frames in flight: it owns their receive buffer.
    ``local`` is this rank's render output for ``frames`` consecutive frames,
    frame f's rows in local order at f * max_rows * w (rows past the rank's
    own are padding and ignored); ``out`` (root only) receives the frames,
    h x w each, back to back.  A group of frames travels as one message.
    ``packed``: the 4-spp binary-shade pixels (5 values, Color + rgbToInt,
    CUDAKernels.cu:384-388,420) travel as 4-bit hit counts, 8 per word --
    8x fewer bytes into the root -- and the root expands them back to the
    same RGBA words (exact: the map is one-to-one on the 5 shades)."""

    def __init__(self, dist, h: int, w: int, band: int, rank: int, world: int, device,
                 root: int = 0, frames: int = 1, packed: bool = False):
        import torch
        self.dist, self.h, self.w, self.rank, self.world, self.root = dist, h, w, rank, world, root
        self.frames = frames
        self.mrows = max_rows(h, band, world)
        self.packed = packed
        n = frames * self.mrows * w
        if packed:
            # 4 spp binary shades: 5 pixel values, 4 bits each, 8 pixels per word
            assert w % 8 == 0, "packed gather needs w % 8 == 0"
            self.k_of_r = torch.full((256,), 15, dtype=torch.int32, device=device)
            self.rgba_of_k = torch.zeros(16, dtype=torch.int32, device=device)
            for k in range(5):
                rg = (255 * k + 20 * (4 - k)) // 4          # CUDAKernels.cu:384-388, :420
                self.k_of_r[rg] = k
                self.rgba_of_k[k] = (10 * (4 - k)) << 16 | rg << 8 | rg
            self.shifts = (4 * torch.arange(8, dtype=torch.int32, device=device)).view(1, 8)
            n //= 8
            self.send = torch.empty(n, dtype=torch.int32, device=device)
        self.n = n
        self.recv = None
        self.parts = None
        self.order = None
        if rank == root:
            self.recv = torch.empty(world * n, dtype=torch.int32, device=device)
            self.parts = [self.recv[r * n:(r + 1) * n] for r in range(world)]
            self.order = torch.from_numpy(gather_order(h, band, world, frames)).to(device)

    def __call__(self, local, out=None):
        import torch
        send = local[: self.frames * self.mrows * self.w]
        if self.packed:
            k = torch.index_select(self.k_of_r, 0, (send & 0xFF).long()).view(-1, 8)
            torch.sum(torch.bitwise_left_shift(k, self.shifts), dim=1, dtype=torch.int32, out=self.send)
            send = self.send
        if self.rank == self.root:
            self.dist.gather(send, self.parts, dst=self.root)
            if out is None:
                return
            rows = self.recv
            if self.packed:
                k = torch.bitwise_and(torch.bitwise_right_shift(self.recv.view(-1, 1), self.shifts), 15)
                rows = torch.index_select(self.rgba_of_k, 0, k.view(-1).long())
            torch.index_select(rows.view(self.world * self.frames * self.mrows, self.w), 0,
                               self.order, out=out[: self.frames * self.h * self.w].view(-1, self.w))
        else:
            self.dist.gather(send, None, dst=self.root)


def frame_of_step(base: int, k: int, rank: int, world: int, group: int = 1) -> int:
    """Frame index rank `rank` renders at its k-th step when whole frames are
    dealt round-robin in groups of `group` consecutive frames: steps k of all
    ranks cover frames base + kN .. base + kN + N-1 (group 1), and a rank's
    group g is frames base + (g N + rank) group + [0, group)."""
    g, j = divmod(k, group)
    return base + (g * world + rank) * group + j
