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


# ---- product-path sharding (vdmi.dist.RecordSink / run_on_devices, pipeline._rank_shard) ----

class _Boxes:
    def __init__(self, frames, cap=3):
        self.count = torch.tensor([f % 4 for f in frames], dtype=torch.int32)
        self.xyxy = torch.tensor([[[f, k, f + 9, k + 9] for k in range(cap)] for f in frames], dtype=torch.int32)
        self.score = torch.tensor([[0.5 + f / 64 + k / 512 for k in range(cap)] for f in frames])
        self.label = torch.tensor([[100 * f + k for k in range(cap)] for f in frames], dtype=torch.int32)


def _expect(f, cap=64, plate=False):
    k = f % 4
    g = (lambda x: x + 1000) if plate else (lambda x: x)
    return ([(g(f), j, g(f) + 9, j + 9) for j in range(min(k, 3))], k)


def test_record_sink_local_rows_and_unpack():
    from vdmi.dist import RecordSink, unpack_sink
    sink = RecordSink(6, cap=64, plates=True)
    sink.add(range(0, 2), range(10, 12), _Boxes([10, 11]), _Boxes([1010, 1011]))
    sink.add([4, 3], [14, 13], _Boxes([14, 13]))                 # out of order rows, no plate lists
    sink.add_lists([5], [15], [[[1.7, 2.2, 30.9, 40.0]]], [[]])  # host lists: int() of float boxes
    got = unpack_sink(sink.gather(), 64, plates=True)
    assert list(got) == [10, 11, 13, 14, 15]                     # row 2 never written, status row skipped
    for f in (10, 11):
        boxes, scores, anchors, count = got[f]["faces"]
        assert (boxes, count) == _expect(f) and anchors == [100 * f + j for j in range(min(f % 4, 3))]
        assert (got[f]["plates"][0], got[f]["plates"][3]) == _expect(f, plate=True)
    assert got[13]["plates"] is None and got[14]["faces"][3] == 2
    assert got[15]["faces"][0] == [(1, 2, 30, 40)] and got[15]["plates"][3] == 0


def test_run_on_devices_order_and_errors():
    from vdmi.dist import run_on_devices
    assert run_on_devices(lambda i, sh: (i, sum(sh)), [[1, 2], [3], []]) == [(0, 3), (1, 3), (2, 0)]
    ran = []

    def fn(i, sh):
        ran.append(i)
        if i == 1:
            raise ValueError("device 1 failed")
        return i
    with pytest.raises(ValueError, match="device 1"):
        run_on_devices(fn, [0, 1, 2])
    assert sorted(ran) == [0, 1, 2]                              # the others still ran to completion


def test_resolve_devices(monkeypatch):
    from vdmi.face import resolve_devices
    monkeypatch.delenv("LOCAL_RANK", raising=False)
    assert resolve_devices([3, 1]) == [3, 1] and resolve_devices(None, 2) == [2]
    monkeypatch.setenv("LOCAL_RANK", "5")
    assert resolve_devices() == [5] and resolve_devices(None, 0) == [0]
    monkeypatch.delenv("LOCAL_RANK")
    assert resolve_devices() == list(range(max(1, torch.cuda.device_count())))   # DataParallel: all visible
    with pytest.raises(ValueError):
        resolve_devices([])


N_LIST = 11


def _fake_local(fail_rank=None):
    """pipeline._local stand-in: frames [first, first + n) 'processed' on the CPU with
    deterministic boxes (no GPU), records as the real one packs them."""
    def local(paths, first, device, want_rec, run):
        from vdmi.dist import RecordSink, world_info
        if fail_rank is not None and world_info()[0] == fail_rank:
            raise OSError("cannot read image")
        sink = RecordSink(len(paths), cap=64, plates=True)
        fr = list(range(first, first + len(paths)))
        sink.add(range(len(paths)), fr, _Boxes(fr), _Boxes([1000 + f for f in fr]))
        return (len(paths), sum(f % 4 for f in fr), 0), sink.rec
    return local


def _rank_worker(rank, world, port, results, fail_rank):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import logging
        from vdmi import pipeline
        from vdmi.dist import unpack_sink
        pipeline._local = _fake_local(fail_rank)
        run = {"face_detector": None, "fused": False, "mosaic_plates": True}
        paths = [f"/frames/{i:03d}.jpg" for i in range(N_LIST)]
        try:
            res, got = pipeline._rank_shard(paths, None, run)
            results[rank] = (res, unpack_sink(got, 64, plates=True))
        except Exception as e:      # noqa: BLE001
            results[rank] = ("raised", type(e).__name__, str(e))
        logging.shutdown()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("fail_rank", [None, 1])
def test_rank_shard_totals_and_failure_two_ranks_gloo(fail_rank):
    """pipeline._rank_shard over two gloo ranks: each takes shard_range of the sorted
    list, ONE all-gather gives every rank the whole list's records and totals; a
    failure on one rank raises on BOTH (the failing rank still joins the collective,
    so nobody hangs)."""
    world = 2
    mgr = mp.Manager()
    results = mgr.dict()
    mp.spawn(_rank_worker, args=(world, _free_port(), results, fail_rank), nprocs=world, join=True)
    if fail_rank is not None:
        assert results[fail_rank][:2] == ("raised", "OSError")
        assert results[1 - fail_rank][:2] == ("raised", "RuntimeError") and "[1]" in results[1 - fail_rank][2]
        return
    plates = sum(min(f % 4, 64) for f in range(1000, 1000 + N_LIST))
    for r in range(world):
        res, got = results[r]
        assert res == (N_LIST, sum(f % 4 for f in range(N_LIST)), plates)
        assert list(got) == list(range(N_LIST))
        for f in range(N_LIST):
            assert (got[f]["faces"][0], got[f]["faces"][3]) == _expect(f)


def test_shard_ranks_without_group_is_a_clear_error(tmp_path):
    """shard="ranks" needs an initialised process group: without one, batch_process_images
    raises a ValueError naming the fix instead of failing inside torch.distributed."""
    from vdmi.pipeline import _shard_mode
    with pytest.raises(ValueError, match="process group"):
        _shard_mode("ranks", object(), None, False)
    assert _shard_mode(None, object(), None, False) == "none"


def test_run_on_devices_binds_devices_only_when_given():
    """run_on_devices(devices=...) checks the device list against the shards; without a
    GPU the device scope is a no-op, so the CPU path runs the same."""
    from vdmi.dist import run_on_devices
    assert run_on_devices(lambda i, sh: i * 10 + sh, [1, 2], devices=[0, 0]) == [1, 12]
    with pytest.raises(ValueError):
        run_on_devices(lambda i, sh: sh, [1, 2], devices=[0])
