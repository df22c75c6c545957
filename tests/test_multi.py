"""N > 1 path on CPU: bench.py's per-rank segment sharding and its only
collectives (record all-gather + wall-time max-reduce), run with the gloo
backend at world size 2 (the GPU box runs the same code over RCCL)."""
import os
import socket
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, ROOT)
    import bench
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        frames = 32 * (rank + 1)
        total, wall, recs = bench.gather_records(frames, 1000 + rank, 0.5 + rank, world, torch.device("cpu"))
        out[rank] = (total, wall, recs, bench.segment_base(rank))
    finally:
        dist.destroy_process_group()


def test_gather_records_gloo_world2():
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    for rank in range(world):
        total, wall, recs, base = out[rank]
        assert total == 32 + 64
        assert wall == pytest.approx(1.5)                 # max over ranks
        assert recs == [(32, 1000), (64, 1001)]
    assert out[0][3] != out[1][3]                          # disjoint segments per rank


def test_gather_records_single():
    sys.path.insert(0, ROOT)
    import bench
    total, wall, recs = bench.gather_records(7, 3, 0.25, 1, torch.device("cpu"))
    assert (total, wall, recs) == (7, 0.25, [(7, 3)])
