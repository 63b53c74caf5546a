"""Multi-rank frame sharding through the real detect+blur path.

Two processes (gloo for the collective, both opening a vd context on cuda:0 --
the one GPU of the test box) shard ONE frame list with vdmi.dist.shard_range,
run vd_process (faces + mosaic) on their shard, and all-gather the per-frame
records (frame index, count, int boxes, scores, anchors) plus a per-frame digest
of the mosaicked pixels. Every rank must then hold exactly what a single process
computes over the whole list. fp32 mode: its kernel choice does not depend on
the batch size, so per-frame results are batch-invariant by construction.
"""
import hashlib
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N_FRAMES, H, W, CAP = 7, 1080, 1920, 64


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _digest(img):
    return int.from_bytes(hashlib.sha256(np.ascontiguousarray(img).tobytes()).digest()[:7], "little")


def _records(ctx, frames, first):
    """vd_process on host frames -> (int32 records [n, 2+6*CAP], int64 pixel digests [n])."""
    import torch
    from vdmi import _lib
    from vdmi.dist import pack_records
    out, faces, _ = ctx.process(frames, flags=_lib.VD_PROC_FACES | _lib.VD_PROC_MOSAIC)
    n = frames.shape[0]
    rec = pack_records(torch.from_numpy(faces.count.copy()), torch.from_numpy(faces.xyxy.copy()), CAP,
                       torch.from_numpy(faces.score.copy()), torch.from_numpy(faces.label.copy()),
                       torch.arange(first, first + n, dtype=torch.int32))
    dig = torch.tensor([_digest(out[i]) for i in range(n)], dtype=torch.int64)
    return rec, dig


def _worker(rank, world, port, results):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "video-desensitization_amd")]
    import torch
    import torch.distributed as dist
    import vdmi
    from vdmi import synth, weights
    from vdmi.dist import all_gather_records, rec_width, shard_range, unpack_records
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        b, e = shard_range(N_FRAMES, world, rank)
        per_rank = -(-N_FRAMES // world)
        ctx = vdmi.Context(device=0, precision="fp32", max_batch=per_rank)
        ctx.load_weights(0, weights.retinaface_state_dict(0))
        rec, dig = _records(ctx, synth.frames(e - b, H, W, seed=0, start=b), b)
        ctx.close()
        if rec.shape[0] < per_rank:                      # uneven shard: padding rows (frame -1)
            pad = torch.zeros((per_rank - rec.shape[0], rec_width(CAP)), dtype=torch.int32)
            pad[:, 0] = -1
            rec = torch.cat([rec, pad])
            dig = torch.cat([dig, torch.full((per_rank - dig.shape[0],), -1, dtype=torch.int64)])
        allrec = all_gather_records(rec)
        parts = [torch.empty_like(dig) for _ in range(world)]
        dist.all_gather(parts, dig)
        alldig = torch.cat(parts)
        got = unpack_records(allrec)
        frames = allrec[:, 0].tolist()
        results[rank] = (got, {f: int(d) for f, d in zip(frames, alldig.tolist()) if f >= 0})
    finally:
        dist.destroy_process_group()


def test_two_ranks_shard_one_list_equal_single_process(gpu):
    import torch.multiprocessing as mp
    import vdmi
    from vdmi import synth, weights
    from vdmi.dist import unpack_records
    # single process over the whole list
    ctx = vdmi.Context(device=0, precision="fp32", max_batch=N_FRAMES)
    ctx.load_weights(0, weights.retinaface_state_dict(0))
    rec, dig = _records(ctx, synth.frames(N_FRAMES, H, W, seed=0), 0)
    ctx.close()
    exp = unpack_records(rec)
    exp_dig = {f: int(d) for f, d in enumerate(dig.tolist())}
    assert sum(v[3] for v in exp.values()) > 0            # faces were found to compare
    world = 2
    mgr = mp.Manager()
    results = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), results), nprocs=world, join=True)
    for r in range(world):
        got, got_dig = results[r]
        assert list(got) == list(range(N_FRAMES))
        assert got == exp, f"rank {r}: gathered records differ from the single-process run"
        assert got_dig == exp_dig, f"rank {r}: mosaicked pixels differ from the single-process run"
