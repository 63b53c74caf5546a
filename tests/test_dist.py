"""Frame sharding + box-record all-gather, exercised with world_size=2 over gloo on CPU
(the same code path runs over RCCL in bench.py on GPUs)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def test_shard_range_partitions():
    from vdmi.dist import shard_range
    for n in (0, 1, 7, 64, 1001):
        for world in (1, 2, 3, 8):
            spans = [shard_range(n, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [e - b for b, e in spans]
            assert max(sizes) - min(sizes) <= 1


def test_pack_unpack_records():
    from vdmi.dist import pack_records, unpack_records
    count = torch.tensor([2, 0, 5], dtype=torch.int32)
    xyxy = torch.arange(3 * 4 * 4, dtype=torch.int32).reshape(3, 4, 4)
    rec = pack_records(count, xyxy, 4)
    assert rec.shape == (3, 17)
    out = unpack_records(rec)
    assert out[0] == [(0, 1, 2, 3), (4, 5, 6, 7)] and out[1] == [] and len(out[2]) == 4   # capped


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, results):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from vdmi.dist import all_gather_records, pack_records, shard_range, unpack_records
        n_frames, B, cap = 10, 5, 3
        b, e = shard_range(n_frames, world, rank)
        assert e - b == B
        # each rank "detects" frame-index-dependent boxes on its own shard
        count = torch.tensor([(f % 4) for f in range(b, e)], dtype=torch.int32)
        xyxy = torch.tensor([[[f, k, f + 10, k + 10] for k in range(cap)] for f in range(b, e)], dtype=torch.int32)
        allrec = all_gather_records(pack_records(count, xyxy, cap))
        results[rank] = unpack_records(allrec)
    finally:
        dist.destroy_process_group()


def test_all_gather_two_ranks_gloo():
    world = 2
    port = _free_port()
    mgr = mp.Manager()
    results = mgr.dict()
    mp.spawn(_worker, args=(world, port, results), nprocs=world, join=True)
    exp = [[(f, k, f + 10, k + 10) for k in range(min(f % 4, 3))] for f in range(10)]
    assert results[0] == exp and results[1] == exp
