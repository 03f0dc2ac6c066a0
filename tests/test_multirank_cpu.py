"""Multi-rank path on CPU (gloo): each rank renders its interleaved row bands
(with the oracle, since there is no GPU here), the bands are all-gathered and
reassembled with the same tiling code bench.py uses on RCCL; the result must
equal a one-process render byte for byte."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT, edge_scenes


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, w, h, band, out_dir):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "bih-gpu-raytracer_amd"))
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import oracle
    from bihrt.tiling import band_rows, gather_order, max_rows, rows_of_rank
    ot = oracle.OracleTree(edge_scenes()["cornell"])
    rows = band_rows(h, band, rank, world)
    ys = rows_of_rank(h, band, rank, world)
    assert rows.nrows == ys.size
    # bih_rows' local -> global row map (include/bih.h) gives the same rows
    lr = np.arange(rows.nrows)
    assert np.array_equal(rows.row0 + (lr // rows.band_h) * rows.band_h * rows.band_step
                          + lr % rows.band_h, ys)
    mrows = max_rows(h, band, world)
    local = np.zeros((mrows, w), np.uint32)
    for k, y in enumerate(ys):
        local[k], _ = ot.render(w, h, rows=(int(y), 1, 1))
    t = torch.from_numpy(local.view(np.int32).reshape(-1))
    parts = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(parts, t)
    gathered = torch.cat(parts).view(world * mrows, w)
    frame = torch.index_select(gathered, 0, torch.from_numpy(gather_order(h, band, world)))
    np.save(os.path.join(out_dir, f"frame_{rank}.npy"), frame.numpy().view(np.uint32))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,band", [(2, 8), (3, 4)])
def test_band_tiling_gather_equals_single_render(tmp_path, world, band, oracle_mod):
    w, h = 48, 40
    mp.start_processes(_worker, args=(world, _free_port(), w, h, band, str(tmp_path)),
                       nprocs=world, join=True, start_method="spawn")
    ref, _ = oracle_mod.OracleTree(edge_scenes()["cornell"]).render(w, h)
    for r in range(world):
        assert np.array_equal(np.load(tmp_path / f"frame_{r}.npy"), ref)
