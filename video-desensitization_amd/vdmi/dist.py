"""Multi-GPU frame sharding: the product path's two forms.

The reference's only multi-GPU mechanism is nn.DataParallel inside one process
(detect_face/face.py:55-56): every forward re-broadcasts ~109 MB of fp32 weights,
scatters the input and gathers (loc, conf, landm) to cuda:0. Here frames are
independent units, so the MI355X design is one process per GPU over
torch.distributed (backend "nccl" = RCCL on ROCm):

* rank r owns the contiguous frame range [r*N/G, (r+1)*N/G) of a video, in
  batches of B; weights are uploaded once per rank; pixels never leave their GPU;
* the only exchange is an all-gather of fixed-size per-frame box records
  ``[frame, count, 64 x (x1, y1, x2, y2), 64 x score, 64 x anchor]`` (int32,
  2 + 6*cap words) over xGMI, so every rank (or the writer) sees the whole
  batch's detections. At cap=64 that is ~1.5 KB per frame, ~100 KB per rank per
  step: latency-bound, far below one xGMI link's ~153 GB/s, so a single ring
  all-gather is the right collective. Uneven shards pad to the largest with
  frame = -1 rows (all_gather_into_tensor needs equal blocks).

Two ways to use every GPU, both used by ``vdmi.pipeline.batch_process_images``:

* **ranks** (``torchrun --nproc-per-node N``; ``init_from_env``): rank r processes
  its contiguous shard of the frame list on its own GPU, packs each frame's record
  on the device right behind the call that produced its boxes (``RecordSink``), and
  the ranks exchange the records once, with one RCCL all-gather (``RecordSink.gather``);
* **devices** (one process, ``run_on_devices``): one context per visible GPU, one
  host thread per device driving it (ctypes releases the GIL during the C calls),
  each device taking a contiguous shard -- the direct replacement for
  ``nn.DataParallel`` without its per-forward replicate / scatter / gather.

``process_frames`` is the device-resident shard loop (frames already in HBM):
``bench.py`` times exactly this function.
"""
import os
import threading

import numpy as np


def shard_range(n_frames, world, rank):
    """Contiguous [begin, end) frame range of `rank` (sizes differ by at most 1)."""
    base, rem = divmod(n_frames, world)
    begin = rank * base + min(rank, rem)
    return begin, begin + base + (1 if rank < rem else 0)


REC_HDR = 2   # words before the boxes: frame index, count


def rec_width(cap):
    """int32 words per frame record: frame, count, cap boxes, cap scores, cap anchors."""
    return REC_HDR + 6 * cap


def pack_records(count, xyxy, cap, score=None, anchor=None, frame=None):
    """int32 [n, 2 + 6*cap] per-frame records: global frame index,
    kept-box count (complete, may exceed cap), then the first `cap` int boxes,
    their f32 scores (bit pattern) and anchor indices. Padding rows use frame -1."""
    import torch
    n = count.shape[0]
    dev = count.device
    rec = torch.zeros((n, rec_width(cap)), dtype=torch.int32, device=dev)
    rec[:, 0] = frame if frame is not None else torch.arange(n, dtype=torch.int32, device=dev)
    rec[:, 1] = count
    k = min(cap, xyxy.shape[1])
    rec[:, 2:2 + 4 * k] = xyxy[:, :k].reshape(n, 4 * k)
    if score is not None:
        rec[:, 2 + 4 * cap:2 + 4 * cap + k] = score[:, :k].contiguous().view(torch.int32)
    if anchor is not None:
        rec[:, 2 + 5 * cap:2 + 5 * cap + k] = anchor[:, :k]
    return rec


def unpack_records(rec):
    """-> {frame: (boxes [(x1, y1, x2, y2)], scores [float], anchors [int], count)} for
    every non-padding record; boxes/scores/anchors hold min(count, cap) entries."""
    rec = rec.cpu().numpy() if hasattr(rec, "cpu") else np.asarray(rec)
    rec = np.ascontiguousarray(rec, np.int32)
    cap = (rec.shape[1] - REC_HDR) // 6
    out = {}
    for r in rec:
        f = int(r[0])
        if f < 0:
            continue
        k = min(int(r[1]), cap)
        boxes = [tuple(int(v) for v in r[2 + 4 * i:6 + 4 * i]) for i in range(k)]
        scores = r[2 + 4 * cap:2 + 4 * cap + k].view(np.float32).tolist()
        anchors = [int(v) for v in r[2 + 5 * cap:2 + 5 * cap + k]]
        out[f] = (boxes, scores, anchors, int(r[1]))
    return dict(sorted(out.items()))


def all_gather_records(rec, group=None):
    """all_gather_into_tensor of equal-shaped per-rank record blocks -> [world*n, W]."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    if rec.device.type == "cuda" and dist.get_backend(group) == "gloo":
        # gloo (CPU tests, bench --backend gloo): gather through host memory
        return all_gather_records(rec.cpu(), group).to(rec.device)
    out = torch.empty((world * rec.shape[0], rec.shape[1]), dtype=rec.dtype, device=rec.device)
    if rec.device.type == "cuda":
        dist.all_gather_into_tensor(out, rec.contiguous(), group=group)
    else:   # gloo has no all_gather_into_tensor on every build: list form
        parts = [torch.empty_like(rec) for _ in range(world)]
        dist.all_gather(parts, rec.contiguous(), group=group)
        out = torch.cat(parts, 0)
    return out


STATUS_FRAME = -2   # the status row every rank appends to its gathered block


def world_info(group=None):
    """(rank, world) of the initialised default / given process group, else (0, 1)."""
    try:
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized():
            return dist.get_rank(group), dist.get_world_size(group)
    except Exception:
        pass
    return 0, 1


def _group_on():
    """A process group is initialised (the collective runs even at world 1: bench.py
    --force-dist exercises the RCCL branch on a one-GPU box)."""
    try:
        import torch.distributed as dist
        return dist.is_available() and dist.is_initialized()
    except Exception:
        return False


def local_device():
    """This process's GPU: LOCAL_RANK under torchrun, else 0 (an env read: no GPU call)."""
    return int(os.environ.get("LOCAL_RANK", "0") or 0)


def init_from_env(backend="nccl", same_device=False):
    """For a rank started by torchrun: bind its GPU (LOCAL_RANK, or cuda:0 with
    same_device -- a one-GPU rehearsal) and join the process group over RCCL
    ("nccl" is RCCL on ROCm; "gloo" for CPU tests / same-device rehearsals).
    Returns (rank, world, device index)."""
    import torch
    import torch.distributed as dist
    dev = 0 if same_device else local_device()
    if not dist.is_initialized():
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{dev}"))
        else:
            dist.init_process_group(backend)
    if torch.cuda.is_available():
        torch.cuda.set_device(dev)
    return dist.get_rank(), dist.get_world_size(), dev


class RecordSink:
    """The per-frame box records of one shard, ``[rows, W]`` int32 (W = rec_width(cap),
    doubled when plate lists ride along: ``[face record | plate record]``), kept where
    the boxes were produced. ``add`` packs a call's boxes on the stream that produced
    them (queued right behind the call, no host wait); ``gather`` exchanges the shard
    blocks of every rank with ONE all-gather (RCCL over xGMI for device tensors) and
    returns the whole list's records on every rank. Rows never written stay
    ``frame = -1`` (a dropped batch, or padding of a short shard)."""

    def __init__(self, rows, cap=64, device=None, plates=False):
        import torch
        self.torch = torch
        self.cap, self.plates, self.rows = int(cap), bool(plates), int(rows)
        self.w = rec_width(self.cap)
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        self.rec = torch.zeros((self.rows, self.w * (2 if plates else 1)), dtype=torch.int32, device=self.device)
        self.rec[:, 0] = -1
        if plates:
            self.rec[:, self.w] = -1
        # the fill above runs on this thread's current stream; add() packs on the stream
        # that produced the boxes, which must not overtake it (an event orders the two)
        self._init_ev = None
        if self.device.type == "cuda":
            self._init_ev = torch.cuda.Event()
            self._init_ev.record(torch.cuda.current_stream(self.device))
        self.lock = threading.Lock()

    def _stream_ctx(self, stream):
        import contextlib
        if stream is None or self.device.type != "cuda":
            return contextlib.nullcontext()
        if isinstance(stream, int):
            stream = self.torch.cuda.ExternalStream(stream, device=self.device)
        return self.torch.cuda.stream(stream)

    def _index(self, seq, dtype):
        """An index list on the sink's device without a host wait: a contiguous range is
        generated there; any other list goes through pinned memory asynchronously (a
        pageable copy would wait for the stream, i.e. for the call that made the boxes)."""
        torch = self.torch
        if isinstance(seq, range) and seq.step == 1:
            return torch.arange(seq.start, seq.stop, dtype=dtype, device=self.device)
        h = torch.as_tensor(list(seq), dtype=dtype)
        if self.device.type != "cuda":
            return h
        return h.pin_memory().to(self.device, non_blocking=True)

    def add(self, rows, frame_ids, faces, plates=None, stream=None):
        """Pack len(rows) frames' boxes (DeviceBoxes / HostBoxes holding exactly those
        frames, in order) into `rows` of the sink with global `frame_ids`. `stream`: the
        stream (torch stream or raw HIP stream pointer) the boxes were written on."""
        torch = self.torch
        n = len(rows)
        if n == 0:
            return
        with self._stream_ctx(stream):
            dev = self.device
            if self._init_ev is not None:
                torch.cuda.current_stream(dev).wait_event(self._init_ev)
            t = lambda a, dt: (a if isinstance(a, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(a))
                               ).to(device=dev, dtype=dt, non_blocking=False)
            ids = self._index(frame_ids, torch.int32)
            r = self._index(rows, torch.int64)
            block = [pack_records(t(faces.count[:n], torch.int32), t(faces.xyxy[:n], torch.int32), self.cap,
                                  t(faces.score[:n], torch.float32), t(faces.label[:n], torch.int32), ids)]
            if self.plates:
                if plates is None:
                    pr = torch.zeros((n, self.w), dtype=torch.int32, device=dev)
                    pr[:, 0] = -1
                else:
                    pr = pack_records(t(plates.count[:n], torch.int32), t(plates.xyxy[:n], torch.int32), self.cap,
                                      t(plates.score[:n], torch.float32), t(plates.label[:n], torch.int32), ids)
                block.append(pr)
            with self.lock:
                self.rec.index_copy_(0, r, torch.cat(block, 1) if len(block) > 1 else block[0])

    def add_lists(self, rows, frame_ids, face_boxes, plate_boxes=None):
        """Host box lists (generic detectors: int boxes only, score 0, anchor -1)."""
        n = len(rows)
        if n == 0:
            return

        class _L:
            pass

        def boxes(lists):
            k = max([len(b) for b in lists] + [1])
            b = _L()
            b.count = np.array([len(x) for x in lists], np.int32)
            b.xyxy = np.zeros((n, k, 4), np.int32)
            for i, x in enumerate(lists):
                if len(x):
                    b.xyxy[i, :len(x)] = np.asarray([[int(v) for v in bb[:4]] for bb in x], np.int32)
            b.score = np.zeros((n, k), np.float32)
            b.label = np.full((n, k), -1, np.int32)
            return b
        self.add(rows, frame_ids, boxes(face_boxes), boxes(plate_boxes) if plate_boxes is not None else None)

    def gather(self, group=None, status=0):
        """All ranks' blocks, plus one status row per rank (frame STATUS_FRAME, count =
        that rank's status: 0 ok, else it failed) -> records [world * (rows + 1), W'],
        queued on the current stream (no host wait; statuses() reads the status rows).
        Every rank of the group must call it (once per sink), with the same `rows`.
        Without a process group: the local block."""
        torch = self.torch
        st = torch.zeros((1, self.rec.shape[1]), dtype=torch.int32, device=self.device)
        st[0, 0], st[0, 1] = STATUS_FRAME, int(status)
        if self.plates:
            st[0, self.w] = -1
        blk = torch.cat([self.rec, st])
        return all_gather_records(blk, group) if _group_on() else blk

    def statuses(self, gathered):
        """Per-rank status of a gather() result (host read: waits for it)."""
        per = self.rows + 1
        return [int(v) for v in gathered[per - 1::per, 1].tolist()]


def unpack_sink(rec, cap=64, plates=False):
    """Gathered RecordSink rows -> {frame: {"faces": (boxes, scores, anchors, count),
    "plates": (...) or None}} for every written frame, in frame order."""
    w = rec_width(cap)
    rec = rec.cpu() if hasattr(rec, "cpu") else rec
    faces = unpack_records(rec[:, :w])
    pl = unpack_records(rec[:, w:2 * w]) if plates else {}
    return {f: {"faces": v, "plates": pl.get(f)} for f, v in faces.items()}


def process_frames(ctx, frames, out, batch, first_frame, sink, flags, faces, plates=None, row0=0):
    """One shard of device-resident frames (torch uint8 [n, h, w, 3] on ctx's GPU) in
    batches of `batch`: one vd_process per batch into `out`, each batch's box records
    packed into `sink` rows [row0 + s, row0 + s + n) with global frame ids
    first_frame + s ..., on the context's stream. faces / plates: DeviceBoxes of at
    least `batch` frames (reused per batch: the record is packed before the next
    batch overwrites them, in stream order). Queued asynchronously; returns the
    number of frames."""
    n_all = frames.shape[0]
    for s in range(0, n_all, batch):
        n = min(batch, n_all - s)
        fv = faces.view(0, n) if faces is not None else None
        pv = plates.view(0, n) if plates is not None else None
        ctx.process(frames[s:s + n], out[s:s + n] if out is not None else None, faces=fv, plates=pv, flags=flags)
        if sink is not None:
            sink.add(range(row0 + s, row0 + s + n), range(first_frame + s, first_frame + s + n), fv, pv,
                     stream=ctx.stream())
    return n_all


def _device_scope(dev):
    """torch.cuda.device(dev) when a GPU is usable (so a tensor, stream or event a
    shard's code creates without naming a device lands on ITS device, not on the
    thread's default cuda:0), else nothing."""
    import contextlib
    if dev is None:
        return contextlib.nullcontext()
    try:
        import torch
        if torch.cuda.is_available():
            return torch.cuda.device(int(dev))
    except Exception:
        pass
    return contextlib.nullcontext()


def run_on_devices(fn, shards, devices=None):
    """Run fn(i, shard) for every shard on its own thread (one per device: each
    drives its own context, whose C calls release the GIL) and wait for all.
    devices[i] (optional): the GPU of shard i; its thread runs fn inside
    torch.cuda.device(devices[i]). Returns the results in shard order; re-raises the
    first shard's exception (in shard order) after every thread has finished."""
    res = [None] * len(shards)
    err = [None] * len(shards)
    if devices is not None and len(devices) != len(shards):
        raise ValueError(f"run_on_devices: {len(devices)} devices for {len(shards)} shards")

    def work(i):
        try:
            with _device_scope(devices[i] if devices is not None else None):
                res[i] = fn(i, shards[i])
        except BaseException as e:           # noqa: B902 -- re-raised below
            err[i] = e

    if len(shards) == 1:
        work(0)
    else:
        th = [threading.Thread(target=work, args=(i,), name=f"vdmi-dev{i}") for i in range(len(shards))]
        for t in th:
            t.start()
        for t in th:
            t.join()
    for e in err:
        if e is not None:
            raise e
    return res
