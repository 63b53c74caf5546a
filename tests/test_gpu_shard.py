"""Frame sharding in the PRODUCT path (the reference's
nn.DataParallel, detect_face/face.py:55-56, splits every forward over all GPUs):

* "devices": one process, one context per device, one host thread each -- here two
  contexts on the one GPU of the test box (device_ids=[0, 0], a same-device
  rehearsal of two GPUs);
* "ranks": torchrun-style ranks, each processing vdmi.dist.shard_range of the frame
  list and exchanging the per-frame box records with one all-gather -- here two
  spawned ranks on cuda:0 with gloo (RCCL needs distinct GPUs; bench.py's RCCL
  branch is exercised at world 1 in test_gpu_bench_dist.py).

Every form must write byte-identical frames and hand back identical box records
and totals to the single-context run over the same frame directory (the fp32 plan
is batch-invariant: a frame's results do not depend on its batch or shard)."""
import io
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N = 9          # frames: shards of 5 / 4, batches of 4 -> a short last batch on each side


def _frame(i):
    from vdmi import synth
    return np.repeat(np.repeat(synth.frame(180, 320, i, seed=5), 2, 0), 2, 1)     # 360x640, faces fire


def _jpeg_dir(d):
    from PIL import Image
    d.mkdir(exist_ok=True)
    for i in range(N):
        b = io.BytesIO()
        Image.fromarray(_frame(i)).save(b, "JPEG", quality=95)
        (d / f"f{i:03d}.jpg").write_bytes(b.getvalue())
    return d


def _detectors(device_ids):
    import vdmi
    from vdmi import weights
    face = vdmi.Retinaface(input_shape=[640, 640, 3], nms_iou=0.4, max_batch=4, device_ids=device_ids,
                           weights=weights.retinaface_state_dict(0))
    plate = vdmi.YOLO(weights="random", max_batch=4, device_ids=device_ids)
    return face, plate


def _files(d):
    return {f: (d / f).read_bytes() for f in sorted(os.listdir(d))}


def test_detect_images_two_contexts_equal_one(gpu):
    """Retinaface / YOLO with two device contexts: the image list is split over them
    (one thread each) and every image's boxes equal the one-context detector's."""
    imgs = [_frame(i) for i in range(5)] + [np.ascontiguousarray(_frame(7)[:300, :500])]
    f1, p1 = _detectors([0])
    f2, p2 = _detectors([0, 0])
    assert len(f2.ctxs) == 2 and len(p2.ctxs) == 2
    a, b = f1.detect_images(imgs), f2.detect_images(imgs)
    assert [x[1] for x in a] == [x[1] for x in b] and sum(len(x[1]) for x in a) > 0
    pa, pb = p1(imgs), p2(imgs)
    for x, y in zip(pa, pb):
        np.testing.assert_array_equal(x.boxes.xyxy, y.boxes.xyxy)
        np.testing.assert_array_equal(x.boxes.conf, y.boxes.conf)


@pytest.mark.parametrize("codec", [True, False])
def test_batch_process_images_devices_equal_single(gpu, tmp_path, codec):
    """shard="devices" (two contexts, one thread each, contiguous shards of the list):
    the written frames (GPU JPEG codec path: file bytes; fused host-frame path: saved
    arrays), the per-frame records and the totals equal the single-context run's."""
    from vdmi.pipeline import batch_process_images
    src = _jpeg_dir(tmp_path / "in")
    kw = {} if codec else {"loader": lambda p: _frame(int(os.path.basename(p)[1:4]))}
    runs = {}
    dets = {"one": _detectors([0]), "two": _detectors([0, 0])}
    # "two" runs twice on the same detectors: the second call finds its fused contexts
    # cached, and each shard must still get its OWN context (ids repeat: [0, 0])
    for name, det, shard in (("one", "one", None), ("two", "two", "devices"), ("two_again", "two", "devices")):
        face, plate = dets[det]
        saved, rec = {}, {}
        if not codec:
            kw["saver"] = lambda img, p, saved=saved: saved.__setitem__(os.path.basename(p), img.copy())
        out = tmp_path / name
        tot = batch_process_images(str(src), str(out), face, plate, batch_size=4, shard=shard, records=rec,
                                   mosaic_plates=True, **kw)
        runs[name] = (tot, rec, _files(out) if codec else saved)
    ctxs = list(dets["two"][0].__dict__["_fused_ctx"].values())
    assert len(ctxs) == 2 and ctxs[0] is not ctxs[1]
    (t1, r1, o1) = runs["one"]
    assert t1[0] == N and t1[1] > 0
    assert sorted(r1) == sorted(o1 if codec else [f"f{i:03d}.jpg" for i in range(N)]) or len(r1) == N
    for name in ("two", "two_again"):
        t2, r2, o2 = runs[name]
        assert t2 == t1 and r2 == r1, name
        assert sorted(o1) == sorted(o2) and len(o1) == N
        for k in o1:
            if codec:
                assert o1[k] == o2[k], (name, k)
            else:
                np.testing.assert_array_equal(o1[k], o2[k], err_msg=f"{name} {k}")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, src, out, results):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), LOCAL_RANK="0", RANK=str(rank),
                      WORLD_SIZE=str(world))
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "video-desensitization_amd"), os.path.join(root, "tests")]
    import torch.distributed as dist
    from vdmi.dist import init_from_env
    init_from_env("gloo", same_device=True)
    try:
        from vdmi.pipeline import batch_process_images
        from test_gpu_shard import _detectors
        face, plate = _detectors(None)           # LOCAL_RANK -> cuda:0
        rec = {}
        tot = batch_process_images(src, out, face, plate, batch_size=4, records=rec, mosaic_plates=True)
        results[rank] = (tot, rec, face.device_ids)
    finally:
        dist.destroy_process_group()


def test_batch_process_images_two_ranks_equal_single(gpu, tmp_path):
    """shard="auto" inside a two-rank process group takes the "ranks" form: each rank
    decodes / processes / encodes its shard of the sorted list on its own context and
    writes those frames; ONE all-gather of the box records gives both ranks the whole
    list's records and totals. Files, records and totals equal the single-context run."""
    import torch.multiprocessing as mp
    from vdmi.pipeline import batch_process_images
    src = _jpeg_dir(tmp_path / "in")
    face, plate = _detectors([0])
    rec1 = {}
    tot1 = batch_process_images(str(src), str(tmp_path / "one"), face, plate, batch_size=4, records=rec1,
                                mosaic_plates=True)
    mgr = mp.Manager()
    results = mgr.dict()
    mp.spawn(_rank, args=(2, _free_port(), str(src), str(tmp_path / "two"), results), nprocs=2, join=True)
    assert tot1[0] == N and tot1[1] > 0
    for r in range(2):
        tot, rec, ids = results[r]
        assert ids == [0] and tot == tot1 and rec == rec1, r
    assert _files(tmp_path / "two") == _files(tmp_path / "one")
