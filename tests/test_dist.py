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
    from vdmi.dist import pack_records, rec_width, unpack_records
    count = torch.tensor([2, 0, 5], dtype=torch.int32)
    xyxy = torch.arange(3 * 4 * 4, dtype=torch.int32).reshape(3, 4, 4)
    score = torch.linspace(0.5, 0.99, 12).reshape(3, 4)
    anchor = torch.arange(100, 112, dtype=torch.int32).reshape(3, 4)
    rec = pack_records(count, xyxy, 4, score, anchor, torch.tensor([7, 8, 9], dtype=torch.int32))
    assert rec.shape == (3, rec_width(4)) == (3, 26)
    out = unpack_records(rec)
    assert list(out) == [7, 8, 9]
    assert out[7][0] == [(0, 1, 2, 3), (4, 5, 6, 7)] and out[8][0] == [] and len(out[9][0]) == 4   # capped
    assert out[7][1] == score[0, :2].tolist() and out[9][2] == [108, 109, 110, 111] and out[9][3] == 5


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
        n_frames, cap = 11, 3                    # uneven shards: 6 + 5 frames, padded to 6
        b, e = shard_range(n_frames, world, rank)
        per_rank = -(-n_frames // world)
        # each rank "detects" frame-index-dependent boxes on its own shard
        count = torch.tensor([(f % 5) for f in range(b, e)], dtype=torch.int32)
        xyxy = torch.tensor([[[f, k, f + 10, k + 10] for k in range(cap)] for f in range(b, e)], dtype=torch.int32)
        score = torch.tensor([[0.5 + f / 100 + k / 1000 for k in range(cap)] for f in range(b, e)])
        anchor = torch.tensor([[f * 10 + k for k in range(cap)] for f in range(b, e)], dtype=torch.int32)
        rec = pack_records(count, xyxy, cap, score, anchor, torch.arange(b, e, dtype=torch.int32))
        if rec.shape[0] < per_rank:
            pad = torch.zeros((per_rank - rec.shape[0], rec.shape[1]), dtype=torch.int32)
            pad[:, 0] = -1
            rec = torch.cat([rec, pad])
        results[rank] = unpack_records(all_gather_records(rec))
    finally:
        dist.destroy_process_group()


def test_all_gather_two_ranks_gloo():
    world = 2
    port = _free_port()
    mgr = mp.Manager()
    results = mgr.dict()
    mp.spawn(_worker, args=(world, port, results), nprocs=world, join=True)
    for r in (0, 1):
        got = results[r]
        assert list(got) == list(range(11))
        for f in range(11):
            k = min(f % 5, 3)
            boxes, scores, anchors, count = got[f]
            assert boxes == [(f, j, f + 10, j + 10) for j in range(k)] and count == f % 5
            assert anchors == [f * 10 + j for j in range(k)]
            np.testing.assert_allclose(scores, [0.5 + f / 100 + j / 1000 for j in range(k)], rtol=1e-6)
