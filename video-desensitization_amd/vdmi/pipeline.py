"""Hot-loop body of the reference driver on the MI355X path.

``batch_process_images`` mirrors combine_detect.py:183-277 (same signature, same
per-batch semantics): list the frame files, load a batch, detect faces and
plates, take face boxes from ``face_results[j][1]`` and plate boxes from
``plate_results[j][1] if isinstance(..., tuple) else []`` (combine_detect.py:237-239
-- Results objects yield [], so plate boxes are discarded exactly as in the
reference unless ``mosaic_plates=True``), int() them (:243-244), mosaic every box
in order (:246-249), save, count, and drop a batch whose inference raises
(:226-228). A frame that fails to load aborts the call, as in the reference (its
loader runs outside the try, :209-211), after the batches already submitted have
been finished and saved.

When both detectors are the vdmi drop-ins, the batch body is ONE ``vd_process``
on one context (letterbox, both forwards, NMS, mosaic of every kept box) driven
by ``FramePipeline``: pinned host buffers, double-buffered device slots and
three HIP streams (host->device copy, compute, device->host copy), so batch
i's upload and batch i-1's download overlap batch i's compute; file decode and
encode run on worker threads beside it. Other detector objects take the
reference's two-thread path unchanged.

File I/O uses cv2 when importable (combine_detect.py:167-180: imread + BGR->RGB,
imwrite of RGB->BGR) and Pillow otherwise; ``loader`` / ``saver`` override both.
"""
import collections
import logging
import os
import threading
from concurrent.futures import ThreadPoolExecutor

import numpy as np

from . import _lib
from .mosaic import mosaic_frames

IMAGE_EXT = (".png", ".jpg", ".jpeg")


def _cv2():
    try:
        import cv2
        return cv2
    except Exception:
        return None


def load_image_rgb(path):
    """combine_detect.py:167-172 (cv2.imread + BGR->RGB); Pillow when cv2 is absent."""
    cv2 = _cv2()
    if cv2 is not None:
        img = cv2.imread(path)
        if img is None:
            raise ValueError(f"cannot read image: {path}")
        return cv2.cvtColor(img, cv2.COLOR_BGR2RGB)
    from PIL import Image
    with Image.open(path) as im:
        return np.asarray(im.convert("RGB"))


def save_output_image(image_array, output_path):
    """combine_detect.py:177-180 (cv2.imwrite, JPEG quality 95 by default); Pillow
    (quality 95) when cv2 is absent."""
    cv2 = _cv2()
    if cv2 is not None:
        cv2.imwrite(output_path, cv2.cvtColor(image_array, cv2.COLOR_RGB2BGR))
        return
    from PIL import Image
    Image.fromarray(np.ascontiguousarray(image_array)).save(output_path, quality=95)


def _boxes_of(result):
    return result[1] if isinstance(result, tuple) else []


class FramePipeline:
    """Pipelined ``vd_process`` over host frame batches on one context.

    Per batch i (slot i % depth): host frames -> pinned slot (CPU copy), then on
    the upload stream an async H2D into the device slot, on the compute stream
    (the context's stream) one vd_process (faces | plates | mosaic) into the
    device output slot, on the download stream the D2H of the mosaicked frames
    and of the box counts / lists. Events order the three streams; a slot is
    reused only after its previous batch's download completed. ``run`` yields
    each batch's results one batch behind the submission, so the next batch's
    upload and compute are already queued while the caller consumes a result.
    """

    def __init__(self, ctx, h, w, max_batch=None, depth=2, plates=True, mosaic_plates=False, cap=256):
        import torch
        self.torch = torch
        self.ctx = ctx
        self.h, self.w = int(h), int(w)
        self.B = int(max_batch or ctx.cfg.max_batch)
        self.depth = max(2, int(depth))
        self.cap = int(cap)
        dev = torch.device(f"cuda:{ctx.device}")
        self.dev = dev
        flags = _lib.VD_PROC_FACES | _lib.VD_PROC_MOSAIC
        if plates:
            flags |= _lib.VD_PROC_PLATES
            if mosaic_plates:
                flags |= _lib.VD_PROC_MOSAIC_PLATES
        self.flags = flags
        self.plates = bool(plates)
        shp = (self.depth, self.B, self.h, self.w, 3)
        self.h_in = torch.empty(shp, dtype=torch.uint8).pin_memory()
        self.h_out = torch.empty(shp, dtype=torch.uint8).pin_memory()
        self.d_in = torch.empty(shp, dtype=torch.uint8, device=dev)
        self.d_out = torch.empty(shp, dtype=torch.uint8, device=dev)
        from .context import DeviceBoxes
        self.d_faces = [DeviceBoxes(self.B, self.cap, dev) for _ in range(self.depth)]
        self.d_plates = [DeviceBoxes(self.B, self.cap, dev) for _ in range(self.depth)] if plates else None
        nb = 2 if plates else 1
        self.h_cnt = torch.empty((self.depth, nb, self.B), dtype=torch.int32).pin_memory()
        self.h_xy = torch.empty((self.depth, nb, self.B, self.cap, 4), dtype=torch.int32).pin_memory()
        self.s_up = torch.cuda.Stream(dev)
        self.s_comp = torch.cuda.Stream(dev)
        self.s_down = torch.cuda.Stream(dev)
        ctx.set_stream(self.s_comp.cuda_stream)
        ev = lambda: [torch.cuda.Event() for _ in range(self.depth)]
        self.ev_up, self.ev_comp, self.ev_down = ev(), ev(), ev()
        self.used = [False] * self.depth
        self.seq = 0

    def next_input(self, n):
        """Pinned host buffer [n,h,w,3] of the next slot, free to be written (a decoder
        can write frames straight into it); then call submit_filled(n)."""
        if n <= 0 or n > self.B:
            raise ValueError(f"batch of {n} outside [1, {self.B}]")
        k = self.seq % self.depth
        if self.used[k]:
            self.ev_down[k].synchronize()        # the slot's previous batch has left the device
        return self.h_in[k, :n].numpy()

    def submit(self, frames):
        """Queue one batch (numpy uint8 [n,h,w,3]) on the three streams; returns a
        ticket for collect(). Raises (VdError / ValueError) when the batch is rejected."""
        frames = np.ascontiguousarray(frames, np.uint8)
        if frames.ndim != 4 or frames.shape[1:] != (self.h, self.w, 3):
            raise ValueError(f"batch {frames.shape} does not fit the pipeline ({self.B}, {self.h}, {self.w}, 3)")
        self.next_input(frames.shape[0])[...] = frames   # host copy into pinned memory
        return self.submit_filled(frames.shape[0])

    def submit_filled(self, n):
        """Queue the batch already written into next_input(n)'s buffer."""
        torch = self.torch
        k = self.seq % self.depth
        with torch.cuda.stream(self.s_up):
            if self.used[k]:
                self.s_up.wait_event(self.ev_comp[k])      # device input slot no longer read
            self.d_in[k, :n].copy_(self.h_in[k, :n], non_blocking=True)
            self.ev_up[k].record(self.s_up)
        self.s_comp.wait_event(self.ev_up[k])
        if self.used[k]:
            self.s_comp.wait_event(self.ev_down[k])
        faces = self.d_faces[k]
        plates = self.d_plates[k] if self.plates else None
        # several pipelines (one per frame size) may share the context: the compute
        # stream that waited on this slot's upload is the one the library must run on
        self.ctx.set_stream(self.s_comp.cuda_stream)
        self.ctx.process(self.d_in[k, :n], self.d_out[k, :n], faces=faces, plates=plates, flags=self.flags)
        self.ev_comp[k].record(self.s_comp)
        with torch.cuda.stream(self.s_down):
            self.s_down.wait_event(self.ev_comp[k])
            self.h_out[k, :n].copy_(self.d_out[k, :n], non_blocking=True)
            self.h_cnt[k, 0, :n].copy_(faces.count[:n], non_blocking=True)
            self.h_xy[k, 0, :n].copy_(faces.xyxy[:n], non_blocking=True)
            if self.plates:
                self.h_cnt[k, 1, :n].copy_(plates.count[:n], non_blocking=True)
                self.h_xy[k, 1, :n].copy_(plates.xyxy[:n], non_blocking=True)
            self.ev_down[k].record(self.s_down)
        self.used[k] = True
        self.seq += 1
        return (k, n)

    def record(self, ticket, sink, rows, frame_ids):
        """Pack a submitted batch's box records into `sink` (vdmi.dist.RecordSink) on the
        compute stream, right behind its vd_process (no host wait)."""
        k, n = ticket
        sink.add(rows, frame_ids, self.d_faces[k].view(0, n),
                 self.d_plates[k].view(0, n) if self.plates else None, stream=self.s_comp)

    def collect(self, ticket):
        """Wait for a submitted batch: (out uint8 [n,h,w,3], face_counts [n], face_boxes,
        plate_counts, plate_boxes). `out` and the boxes are views of pinned buffers,
        valid until `depth` more batches are submitted. Counts are complete (they may
        exceed cap; the mosaic always covers every kept box)."""
        k, n = ticket
        self.ev_down[k].synchronize()
        cnt = self.h_cnt[k].numpy()
        xy = self.h_xy[k].numpy()
        out = self.h_out[k, :n].numpy()
        faces = [xy[0, j, :min(int(cnt[0, j]), self.cap)] for j in range(n)]
        plates = [xy[1, j, :min(int(cnt[1, j]), self.cap)] for j in range(n)] if self.plates else [None] * n
        return out, cnt[0, :n].copy(), faces, (cnt[1, :n].copy() if self.plates else None), plates

    def run(self, batches):
        """Yield collect() of every batch, one batch behind the submission, so the next
        batch's upload and compute are queued while the caller consumes a result."""
        pending = None
        for frames in batches:
            cur = self.submit(frames)
            if pending is not None:
                yield self.collect(pending)
            pending = cur
        if pending is not None:
            yield self.collect(pending)

    def close(self):
        self.torch.cuda.synchronize(self.dev)
        self.ctx.set_stream(None)


class GpuJpegStages:
    """JPEG frames in, JPEG frames out, three stages in flight on three contexts.

    Job i (slot i % depth): decode on a weight-less context (decode thread; device
    entropy decode + HIP IDCT into the device frame slot), one vd_process on the
    caller's context (faces | plates | mosaic, caller thread), encode on a third
    context (encode thread; HIP FDCT + device Huffman coding). The stages are chained
    by HIP events on the contexts' streams, not by host waits on the device:

        decode(i)  --ev_dec-->  process(i)  --ev_proc-->  encode(i)
        process(i) --ev_proc--> decode(i + depth)   (its input slot is free again)

    so process(i + 1) is queued behind process(i) as soon as decode(i + 1)'s host
    stages are done, and the GPU runs the three contexts' kernels side by side. The
    caller thread waits only on host futures: decode(i) queued, and encode(i - depth)
    finished before process(i) reuses its output slot and box lists.
    combine_detect.py:204-262 is the loop this replaces (cv2.imread -> detect ->
    mosaic -> cv2.imwrite per batch)."""

    SERIAL_PASSES = 6

    def __init__(self, ctx, max_batch, flags, quality=95, subsampling=2, depth=3, cap=256, codec_options=None,
                 decode_overlap=True):
        import torch
        # decode_overlap: True (default) = decode(i + 1) runs beside process(i); False =
        # decode(i + 1) starts once process(i) has finished (device order decode, process,
        # decode, ...; encode still overlaps); "auto" = serial after a decode that needed
        # more than SERIAL_PASSES resynchronisation passes (noise-like entropy data), else
        # overlapped. Serial measured level on 2.4-MB noise frames (792-809 vs 800-825
        # frames/s): the decode stage costs ~50 ms per 64 such frames even with the GPU
        # to itself, ~70 ms beside process
        self.decode_overlap = decode_overlap
        self.last_passes = 0
        self.proc_queued = {}                           # job i -> Event: process(i) is queued (main thread creates)
        self.serial_jobs = 0
        from .context import Context, DeviceBoxes
        self.torch = torch
        self.ctx = ctx
        self.B = int(max_batch)
        self.flags = flags
        self.quality, self.subsampling = int(quality), int(subsampling)
        self.depth = max(2, int(depth))
        dev = self.dev = torch.device(f"cuda:{ctx.device}")
        # codec_options: vd_set_option switches of both codec contexts (jdec_* / jenc_*)
        self.dctx = Context(device=ctx.device, precision="fp32", max_batch=self.B, options=codec_options)
        self.ectx = Context(device=ctx.device, precision="fp32", max_batch=self.B, options=codec_options)
        # the codec contexts run on high-priority streams: their small, latency-bound
        # kernels (entropy-decode passes between host convergence checks) are dispatched
        # ahead of the queued workgroups of the process context's convs
        hi = torch.cuda.Stream.priority_range()[1]
        self.s_dec = torch.cuda.Stream(device=dev, priority=hi)
        self.s_enc = torch.cuda.Stream(device=dev, priority=hi)
        self.dctx.set_stream(self.s_dec.cuda_stream)
        self.ectx.set_stream(self.s_enc.cuda_stream)
        self.faces = [DeviceBoxes(self.B, cap, dev) for _ in range(self.depth)]
        self.plates = [DeviceBoxes(self.B, cap, dev) for _ in range(self.depth)]
        self.ev_dec = [torch.cuda.Event() for _ in range(self.depth)]
        self.ev_proc = [torch.cuda.Event() for _ in range(self.depth)]
        self.buf = {}                                   # (h, w) -> ([d_in] * depth, [d_out] * depth)
        self.dpool, self.epool = ThreadPoolExecutor(1), ThreadPoolExecutor(1)
        self.stats = {"decode_wait": 0.0, "encode_wait": 0.0, "queue": 0.0, "decode": 0.0, "encode": 0.0,
                      "decode_fetch": 0.0, "decode_call": 0.0}

    def _buffers(self, h, w):
        if (h, w) not in self.buf:
            t = self.torch
            mk = lambda: [t.empty((self.B, h, w, 3), dtype=t.uint8, device=self.dev) for _ in range(self.depth)]
            self.buf[(h, w)] = (mk(), mk())
        return self.buf[(h, w)]

    def _decode(self, i, fetch, fallback, wait_ev):
        """-> [(frame indices, h, w)] per frame size of job i, decoded into slot i % depth."""
        import time
        from .context import jpeg_info
        t0 = time.perf_counter()
        blobs = fetch()
        t_f = time.perf_counter()
        groups = {}
        for k, b in enumerate(blobs):
            try:
                key = jpeg_info(b)[:2]
            except Exception:
                if fallback is None:
                    raise
                key = fallback(k).shape[:2]
            groups.setdefault(key, []).append(k)
        if wait_ev is not None:
            self.s_dec.wait_event(wait_ev)              # process(i - depth) is done with the slot
        serial = self.decode_overlap is False or (self.decode_overlap == "auto" and
                                                  self.last_passes > self.SERIAL_PASSES)
        ev = self.proc_queued.get(i - 1) if i > 0 else None
        if serial and ev is not None:
            ev.wait()                                   # process(i - 1) queued (or the run ended)
            self.s_dec.wait_event(self.ev_proc[(i - 1) % self.depth])
            self.serial_jobs += 1
        slot = i % self.depth
        out = []
        t_c = time.perf_counter()
        for (h, w), idx in groups.items():
            din = self._buffers(h, w)[0][slot][:len(idx)]
            try:
                self.dctx.jpeg_decode([blobs[k] for k in idx], out=din)
            except Exception:                           # not a layout the GPU decoder takes: host decode
                if fallback is None:
                    raise
                host = np.stack([fallback(k) for k in idx])
                with self.torch.cuda.stream(self.s_dec):
                    din.copy_(self.torch.from_numpy(host))
            out.append((idx, h, w))
        self.ev_dec[slot].record(self.s_dec)
        self.last_passes = self.dctx.jdec_passes()
        t1 = time.perf_counter()
        self.stats["decode"] += t1 - t0
        self.stats["decode_fetch"] += t_f - t0            # reading the files (the caller's fetch)
        self.stats["decode_call"] += t1 - t_c             # vd_jpeg_decode (host parse, staging, passes)
        return out

    def _encode(self, i, groups):
        """-> [(frame indices, JPEG views)], face / plate counts of job i."""
        import time
        t0 = time.perf_counter()
        slot = i % self.depth
        self.s_enc.wait_event(self.ev_proc[slot])
        res, nf, npl = [], 0, 0
        for idx, h, w, off in groups:
            if idx is None:
                continue
            jp = self.ectx.jpeg_encode(self._buffers(h, w)[1][slot][:len(idx)], quality=self.quality,
                                       subsampling=self.subsampling, copy=False)
            res.append((idx, jp))
        for idx, h, w, off in groups:                   # the encode synchronised: process(i) is complete
            if idx is not None:                         # each size group's own rows of the slot's lists
                nf += int(self.faces[slot].count[off:off + len(idx)].sum().item())
                npl += int(self.plates[slot].count[off:off + len(idx)].sum().item())
        self.stats["encode"] += time.perf_counter() - t0
        return res, nf, npl

    def run(self, jobs, done, on_error=None, on_processed=None):
        """jobs: iterable of (key, fetch, fallback): fetch() -> list of JPEG bytes;
        fallback(k) -> host-decoded RGB frame k or None. done(key, [(frame indices,
        JPEG views)], faces, plates) is called in order on the caller thread. A fetch /
        decode error propagates after every job already processed has been encoded
        and handed to done; a process error drops that job (on_error(key, exc)).
        on_processed(key, frame indices, faces, plates, stream): called on the caller
        thread right after each size group's vd_process is queued, with DeviceBoxes
        views holding exactly that group's frames and the context stream they are
        written on (record packing, vdmi.dist.RecordSink.add)."""
        import collections
        import time
        jobs = iter(jobs)
        dec = collections.deque()                       # (i, key, future)
        enc = collections.deque()                       # (i, key, future)
        nxt = [0]
        D = self.depth

        def submit_decode():
            job = next(jobs, None)
            if job is None:
                return
            key, fetch, fallback = job
            i = nxt[0]
            nxt[0] += 1
            self.proc_queued.setdefault(i, threading.Event())
            self.proc_queued.pop(i - D - 1, None)         # long done
            wait_ev = self.ev_proc[i % D] if i >= D else None
            dec.append((i, key, self.dpool.submit(self._decode, i, fetch, fallback, wait_ev)))

        def finish_one():
            i, key, fut = enc.popleft()
            t = time.perf_counter()
            res, nf, npl = fut.result()
            self.stats["encode_wait"] += time.perf_counter() - t
            done(key, res, nf, npl)

        try:
            submit_decode()
            submit_decode()
            while dec:
                i, key, fut = dec.popleft()
                t = time.perf_counter()
                groups = fut.result()                   # a fetch / decode failure propagates
                t1 = time.perf_counter()
                self.stats["decode_wait"] += t1 - t
                while enc and enc[0][0] <= i - D:       # encode(i - depth) frees the output slot
                    finish_one()
                t2 = time.perf_counter()
                slot = i % D
                self.ctx.stream_wait_event(self.ev_dec[slot])
                ok = []
                off = 0                                 # size groups write their own box-list rows
                for idx, h, w in groups:
                    din, dout = self._buffers(h, w)
                    n = len(idx)
                    try:
                        fv, pv = self.faces[slot].view(off, n), self.plates[slot].view(off, n)
                        self.ctx.process(din[slot][:n], dout[slot][:n], faces=fv, plates=pv, flags=self.flags)
                        if on_processed is not None:
                            on_processed(key, idx, fv, pv, self.ctx.stream())
                        ok.append((idx, h, w, off))
                    except Exception as e:              # combine_detect.py:226-228: the batch is dropped
                        if on_error is None:
                            raise
                        on_error(key, e)
                        ok.append((None, h, w, off))
                    off += n
                self.ev_proc[slot].record(self.torch.cuda.ExternalStream(self.ctx.stream(), device=self.dev))
                self.proc_queued[i].set()
                self.stats["queue"] += time.perf_counter() - t2
                enc.append((i, key, self.epool.submit(self._encode, i, ok)))
                submit_decode()
        finally:
            for _, _, fut in dec:                        # decodes queued behind a failure: not processed
                fut.cancel()
            for ev in list(self.proc_queued.values()):   # release a decode waiting on a job never processed
                ev.set()
            while enc:
                finish_one()
            for _, _, fut in dec:
                try:
                    fut.exception()                      # cancelled or finished: nothing left on the thread
                except Exception:
                    pass
            self.proc_queued.clear()

    def close(self):
        self.dpool.shutdown()
        self.epool.shutdown()
        self.torch.cuda.synchronize(self.dev)
        self.dctx.close()
        self.ectx.close()


_FUSED_LOCK = threading.Lock()


def fused_context(face_detector, plate_detector, batch_size, device=None, slot=0):
    """One context on `device` (default: the face detector's first device) holding both
    drop-ins' weights and the face detector's knobs, cached on the face detector per
    (plate detector, batch size, device, slot). `slot` is the shard index in
    shard="devices" mode: two shards never share a context (its stream and staging are
    per call sequence), also when device ids repeat (device_ids=[0, 0])."""
    from .context import Context
    fd, pd = face_detector, plate_detector
    dev = fd.device_ids[0] if device is None else int(device)
    key = (id(plate_detector), int(batch_size), dev, int(slot))
    with _FUSED_LOCK:
        cache = fd.__dict__.setdefault("_fused_ctx", {})
        if key in cache:
            return cache[key]
        ctx = _new_fused_context(fd, pd, batch_size, dev)
        cache[key] = ctx
        return ctx


def _new_fused_context(fd, pd, batch_size, dev):
    from .context import Context
    ctx = Context(device=dev, precision=fd.precision, max_batch=max(int(batch_size), 1),
                  input_shape=fd.input_shape[:2], confidence=fd.confidence, nms_iou=fd.nms_iou,
                  max_boxes=fd.max_boxes, plate_nc=pd.nc, plate_conf=pd.ctx.cfg.plate_conf,
                  plate_iou=pd.ctx.cfg.plate_iou, plate_max_det=pd.ctx.cfg.plate_max_det,
                  plate_imgsz=pd.ctx.cfg.plate_imgsz, options=getattr(fd, "options", None))
    ctx.load_weights(_lib.VD_NET_RETINAFACE, fd.state_dict)
    ctx.load_weights(_lib.VD_NET_YOLOV8N, pd.state_dict)
    return ctx


def _is_vdmi_pair(face_detector, plate_detector):
    from .face import Retinaface
    from .plate import YOLO
    return isinstance(face_detector, Retinaface) and isinstance(plate_detector, YOLO)


def _shard_mode(shard, face_detector, group, fused):
    """"ranks" (one shard per rank of an initialised process group), "devices" (one
    shard per device of the vdmi face detector, one thread each) or "none"."""
    from .dist import world_info
    if shard in (None, False, "none"):
        return "none"
    _, world = world_info(group)
    if shard == "ranks":
        from .dist import _group_on
        if not _group_on():
            raise ValueError("shard='ranks' needs an initialised torch.distributed process group "
                             "(vdmi.dist.init_from_env under torchrun)")
        return "ranks"
    if shard == "devices":
        if not fused:
            raise ValueError("shard='devices' needs the vdmi Retinaface / YOLO drop-ins")
        return "devices"
    if shard != "auto":
        raise ValueError(f"shard must be 'auto', 'ranks', 'devices' or None, got {shard!r}")
    if world > 1:
        return "ranks"
    if fused and len(getattr(face_detector, "device_ids", [0])) > 1:
        return "devices"
    return "none"


def batch_process_images(input_dir, output_dir, face_detector, plate_detector, batch_size=16,
                         loader=None, saver=None, mosaic_plates=False, mosaic_level=8, num_workers=6,
                         gpu_codec="auto", jpeg_quality=95, shard="auto", group=None, records=None):
    """combine_detect.py:183-277. Returns (total_processed, total_faces, total_plates).

    gpu_codec ("auto" | True | False): with vdmi detectors, no custom loader/saver and
    only .jpg/.jpeg frames (what the reference's ffmpeg split writes), the frames are
    read as bytes, decoded on the GPU (vd_jpeg_decode), processed and encoded on the
    GPU (vd_jpeg_encode, cv2.imwrite's quality 95 / 4:2:0), so pixels never cross
    PCIe; the bytes written equal libjpeg-turbo's encode of the processed frames.

    shard: how the frames use several GPUs (the reference's nn.DataParallel,
    face.py:55-56, splits every forward over all of them):
      "auto"    "ranks" inside an initialised torch.distributed group of more than one
                rank (torchrun), else "devices" when the vdmi face detector holds more
                than one device (Retinaface(device_ids=...); by default every visible
                GPU outside torchrun), else one device;
      "ranks"   the frame list (sorted: every rank sees the same order) is cut into
                contiguous shards, rank r processes vdmi.dist.shard_range(n, world, r)
                on its own GPU and writes those frames, and the ranks exchange the
                per-frame box records with one RCCL all-gather over xGMI (pixels never
                leave their GPU); the returned totals cover the WHOLE list, identical
                on every rank; a failure on any rank raises on every rank;
      "devices" one process, one context and one host thread per device, each device
                taking a contiguous shard of the frame list; totals summed;
      None      one device.
    records: an optional dict, filled with every frame's boxes as
    {file name: {"faces": (int boxes, scores, anchors, count), "plates": ... or None}}
    (vdmi.dist.unpack_sink; the gathered records in "ranks" mode, so every rank gets
    the whole list's)."""
    logger = logging.getLogger("VideoProcessor.batch_process_images")
    custom_io = loader is not None or saver is not None
    if gpu_codec is True and custom_io:
        raise ValueError("gpu_codec=True reads and writes JPEG bytes itself: it cannot use a custom loader/saver")
    loader = loader or load_image_rgb
    saver = saver or save_output_image
    image_paths = [os.path.join(input_dir, f) for f in os.listdir(input_dir) if f.lower().endswith(IMAGE_EXT)]
    os.makedirs(output_dir, exist_ok=True)
    fused = _is_vdmi_pair(face_detector, plate_detector) and mosaic_level == face_detector.ctx.cfg.mosaic_level
    all_jpeg = all(p.lower().endswith((".jpg", ".jpeg")) for p in image_paths)
    codec = fused and gpu_codec and (gpu_codec is True or (not custom_io and all_jpeg))
    mode = _shard_mode(shard, face_detector, group, fused)
    run = dict(output_dir=output_dir, face_detector=face_detector, plate_detector=plate_detector,
               batch_size=batch_size, loader=loader, saver=saver, mosaic_plates=mosaic_plates,
               mosaic_level=mosaic_level, num_workers=num_workers, fused=fused, codec=codec,
               jpeg_quality=jpeg_quality, logger=logger)
    want_rec = records is not None or mode == "ranks"
    if mode == "ranks":
        res, rec = _rank_shard(sorted(image_paths), group, run)
    elif mode == "devices":
        devs = list(face_detector.device_ids)
        from .dist import run_on_devices, shard_range
        spans = [shard_range(len(image_paths), len(devs), i) for i in range(len(devs))]

        def one(i, span):
            b, e = span
            return _local(image_paths[b:e], b, devs[i], want_rec, run, slot=i)
        outs = run_on_devices(one, spans, devices=devs)
        res = tuple(sum(o[0][k] for o in outs) for k in range(3))
        rec = _concat_records([o[1] for o in outs]) if want_rec else None
    else:
        res, rec = _local(image_paths, 0, None, want_rec, run)
    if records is not None and rec is not None:
        from .dist import unpack_sink
        order = sorted(image_paths) if mode == "ranks" else image_paths   # what the frame ids index
        for f, v in unpack_sink(rec, _REC_CAP, True).items():
            records[os.path.basename(order[f])] = v
    logger.info(f"processed {res[0]} images: {res[1]} faces, {res[2]} plates")
    return res


_REC_CAP = 64          # boxes per frame carried in a record (vdmi.dist; counts stay complete)


def _concat_records(recs):
    import torch
    return torch.cat([r.cpu() for r in recs if r is not None]) if any(r is not None for r in recs) else None


def _local(paths, first, device, want_rec, run, slot=0):
    """One device over `paths` (global frame ids first, first + 1, ...): the fused /
    GPU-codec / generic loop; `slot`: the shard's own fused context (devices mode).
    Returns ((processed, faces, plates), records or None)."""
    from .dist import RecordSink
    fd = run["face_detector"]
    io = ThreadPoolExecutor(max_workers=run["num_workers"])
    sink = None
    if want_rec:
        dev = None
        if run["fused"]:
            dev = f"cuda:{fd.device_ids[0] if device is None else device}"
        sink = RecordSink(len(paths), cap=_REC_CAP, device=dev, plates=True)
    ids = {p: (k, first + k) for k, p in enumerate(paths)}
    bs = run["batch_size"]
    batches = [paths[i:i + bs] for i in range(0, len(paths), bs)]
    try:
        if run["fused"] and run["codec"]:
            res = _gpu_codec_batches(batches, run["output_dir"], fd, run["plate_detector"], bs,
                                     run["mosaic_plates"], io, run["logger"], run["jpeg_quality"], device, sink, ids,
                                     slot)
        elif run["fused"]:
            res = _fused_batches(batches, run["output_dir"], fd, run["plate_detector"], bs, run["loader"],
                                 run["saver"], run["mosaic_plates"], io, run["logger"], device, sink, ids, slot)
        else:
            res = _threaded_batches(batches, run["output_dir"], fd, run["plate_detector"], run["loader"],
                                    run["saver"], run["mosaic_plates"], run["mosaic_level"], io, run["logger"],
                                    sink, ids)
    finally:
        io.shutdown(wait=True)
    if sink is not None and sink.device.type == "cuda":
        import torch
        torch.cuda.synchronize(sink.device)
    return res, (sink.rec if sink is not None else None)


def _rank_shard(paths, group, run):
    """This rank's contiguous shard of the (sorted) list through _local, then ONE
    all-gather of the box records of every rank (RCCL for device records). Totals and
    records cover the whole list on every rank. Every rank reaches the all-gather,
    also after a failure of its own (status row), so no rank is left waiting in the
    collective; then every rank raises."""
    from .dist import RecordSink, shard_range, world_info
    rank, world = world_info(group)
    n = len(paths)
    b, e = shard_range(n, world, rank)
    per = -(-n // world) if n else 0
    fd = run["face_detector"]
    err, res, rec = None, (0, 0, 0), None
    try:
        res, rec = _local(paths[b:e], b, None, True, run)
    except Exception as ex:      # noqa: BLE001 -- re-raised after the collective
        err = ex
    dev = f"cuda:{fd.device_ids[0]}" if run["fused"] else None
    if dev is None:
        import torch.distributed as dist
        if dist.get_backend(group) == "nccl":     # RCCL gathers device tensors only
            from .dist import local_device
            dev = f"cuda:{local_device()}"
    sink = RecordSink(per, cap=_REC_CAP, device=dev, plates=True)
    if rec is not None and rec.shape[0]:
        sink.rec[:rec.shape[0]] = rec.to(sink.device)
    got = sink.gather(group, status=0 if err is None else 1)
    status = sink.statuses(got)
    if err is not None:
        raise err
    bad = [r for r, v in enumerate(status) if v]
    if bad:
        raise RuntimeError(f"batch_process_images: rank(s) {bad} failed; their shards are incomplete")
    got = got.cpu()
    w = got.shape[1] // 2
    ok = got[:, 0] >= 0
    total = int(ok.sum())
    faces = int(got[ok, 1].sum())
    plates = int(got[ok, w + 1].clamp(min=0).sum()) if run["mosaic_plates"] else 0
    return (total, faces, plates), got


def _save_all(futs, logger):
    for f in futs:
        try:
            f.result()
        except Exception as e:
            logger.error(f"saving failed: {e}")


def _fused_batches(batches, output_dir, face_detector, plate_detector, batch_size, loader, saver, mosaic_plates,
                   io, logger, device=None, sink=None, ids=None, slot=0):
    """The vdmi path, streaming: decode batch b+1 (threads) while batch b is on the
    GPU (FramePipeline: one vd_process per batch), collect batch b-1 and hand its
    frames to the encoder threads. Frames of another size get their own pipeline;
    a batch whose inference fails is dropped (combine_detect.py:226-228), a load
    failure aborts the call (:209-211). sink / ids: box records packed per batch on
    the compute stream (vdmi.dist.RecordSink; ids: path -> (row, frame id))."""
    totals = [0, 0, 0]
    save_futs = []
    ctx = fused_context(face_detector, plate_detector, batch_size, device, slot)
    pipes = {}
    load = lambda files: list(io.map(loader, files))

    def finish(p):
        pipe, ticket, files = p
        try:
            out, fcnt, _, pcnt, _ = pipe.collect(ticket)
        except Exception as e:           # a fault surfacing at the sync: the batch is dropped
            logger.error(f"parallel inference failed: {e}")
            return
        for path, img in zip(files, out):
            dst = os.path.join(output_dir, f"processed_{os.path.basename(path)}")
            save_futs.append(io.submit(saver, img.copy(), dst))
        totals[0] += len(files)
        totals[1] += int(fcnt.sum())
        if mosaic_plates:                # the reference's tuple check discards plate boxes otherwise
            totals[2] += int(pcnt.sum())

    pending = None
    fut = io.submit(load, batches[0]) if batches else None
    try:
        for bi, files in enumerate(batches):
            imgs = fut.result()          # a load failure propagates (combine_detect.py:209-211)
            fut = io.submit(load, batches[bi + 1]) if bi + 1 < len(batches) else None
            pending = _submit_groups(files, imgs, pipes, ctx, batch_size, mosaic_plates, pending, finish, logger,
                                     sink, ids)
    finally:
        if fut is not None:
            fut.cancel()
        if pending is not None:
            finish(pending)
        for pipe in pipes.values():
            pipe.close()
        _save_all(save_futs, logger)
    return tuple(totals)


def _submit_groups(files, imgs, pipes, ctx, batch_size, mosaic_plates, pending, finish, logger, sink=None, ids=None):
    """Submit one loaded batch (one pipeline per frame size), finishing the previous
    submission behind it; returns the new pending submission."""
    groups = {}
    for f, im in zip(files, imgs):
        groups.setdefault(im.shape, []).append((f, im))
    for shape, items in groups.items():
        if shape not in pipes:
            pipes[shape] = FramePipeline(ctx, shape[0], shape[1], max_batch=batch_size, plates=True,
                                         mosaic_plates=mosaic_plates)
        try:
            pipe = pipes[shape]
            ticket = pipe.submit(np.stack([im for _, im in items]))
            if sink is not None:
                pipe.record(ticket, sink, [ids[f][0] for f, _ in items], [ids[f][1] for f, _ in items])
            cur = (pipe, ticket, [f for f, _ in items])
        except Exception as e:       # combine_detect.py:226-228: the batch is dropped
            logger.error(f"parallel inference failed: {e}")
            cur = None
        if pending is not None:
            finish(pending)
        pending = cur
    return pending


def _read_bytes(path):
    with open(path, "rb") as f:
        return f.read()


def _write_bytes(data, path):
    with open(path, "wb") as f:
        f.write(data)


def _gpu_codec_batches(batches, output_dir, face_detector, plate_detector, batch_size, mosaic_plates, io, logger,
                       quality, device=None, sink=None, ids=None, slot=0):
    """Frame I/O on the GPU (GpuJpegStages): file bytes (reader threads) ->
    vd_jpeg_decode into device frames -> one vd_process (faces | plates | mosaic) ->
    vd_jpeg_encode from device memory -> writer threads, the three stages of
    consecutive batches in flight together, chained by events. A frame the GPU
    decoder does not take (progressive, other layout) is decoded by the host loader;
    a batch whose inference fails is dropped (combine_detect.py:226-228); a read
    failure aborts the call after the batches before it are written (:209-211)."""
    ctx = fused_context(face_detector, plate_detector, batch_size, device, slot)
    flags = _lib.VD_PROC_FACES | _lib.VD_PROC_MOSAIC | _lib.VD_PROC_PLATES
    if mosaic_plates:
        flags |= _lib.VD_PROC_MOSAIC_PLATES
    totals = [0, 0, 0]
    save_futs = []

    def job(files):
        return (files, lambda: list(io.map(_read_bytes, files)), lambda k: load_image_rgb(files[k]))

    def done(files, res, nf, npl):
        for idx, jpegs in res:
            for k, data in zip(idx, jpegs):
                dst = os.path.join(output_dir, f"processed_{os.path.basename(files[k])}")
                save_futs.append(io.submit(_write_bytes, data, dst))
            totals[0] += len(idx)
        totals[1] += nf
        if mosaic_plates:                # the reference's tuple check discards plate boxes otherwise
            totals[2] += npl

    def processed(files, idx, faces, plates, stream):
        sink.add([ids[files[k]][0] for k in idx], [ids[files[k]][1] for k in idx], faces, plates, stream=stream)

    stages = GpuJpegStages(ctx, max(int(batch_size), 1), flags, quality=quality, subsampling=2)
    try:
        stages.run((job(files) for files in batches), done,
                   on_error=lambda files, e: logger.error(f"parallel inference failed: {e}"),
                   on_processed=processed if sink is not None else None)
    finally:
        stages.close()
        _save_all(save_futs, logger)
    return tuple(totals)


def _threaded_batches(batches, output_dir, face_detector, plate_detector, loader, saver, mosaic_plates,
                      mosaic_level, io, logger, sink=None, ids=None):
    """Generic detectors: the reference's two-thread face || plate submission, then
    one batched mosaic launch per same-size group."""
    total = faces = plates = 0
    save_futs = []
    for files in batches:
        batch_images = list(io.map(loader, files))      # raises, as combine_detect.py:209-211
        with ThreadPoolExecutor(max_workers=2) as infer:   # face || plate, as the reference does
            ff = infer.submit(face_detector.detect_images, batch_images.copy())
            fp = infer.submit(plate_detector, batch_images.copy(), verbose=False, conf=0.5)
            try:
                face_results = ff.result()
                plate_results = fp.result()
            except Exception as e:   # combine_detect.py:226-228: the batch is dropped
                logger.error(f"parallel inference failed: {e}")
                continue
        per_frame = []
        fl, pl = [], []
        for j in range(len(batch_images)):
            face_boxes = _boxes_of(face_results[j])
            if mosaic_plates and not isinstance(plate_results[j], tuple):
                plate_boxes = plate_results[j].boxes.xyxy.tolist()
            else:
                plate_boxes = _boxes_of(plate_results[j])
            boxes = [(int(x1), int(y1), int(x2), int(y2)) for x1, y1, x2, y2 in face_boxes]
            boxes += [(int(x1), int(y1), int(x2), int(y2)) for x1, y1, x2, y2 in plate_boxes]
            per_frame.append(boxes)
            fl.append(face_boxes)
            pl.append(plate_boxes)
            faces += len(face_boxes)
            plates += len(plate_boxes)
        if sink is not None:
            sink.add_lists([ids[f][0] for f in files], [ids[f][1] for f in files], fl, pl)
        processed = _mosaic_grouped(batch_images, per_frame, mosaic_level)
        for path, img in zip(files, processed):
            out = os.path.join(output_dir, f"processed_{os.path.basename(path)}")
            save_futs.append(io.submit(saver, img, out))
        total += len(files)
    _save_all(save_futs, logger)
    return total, faces, plates


def _mosaic_grouped(images, boxes, level):
    """One mosaic launch per same-size group of frames."""
    out = [None] * len(images)
    groups = {}
    for i, im in enumerate(images):
        groups.setdefault(im.shape, []).append(i)
    for idx in groups.values():
        res = mosaic_frames(np.stack([images[i] for i in idx]), [boxes[i] for i in idx], level)
        for k, i in enumerate(idx):
            out[i] = res[k]
    return out


def process_batch(ctx, frames, out=None, faces=None, plates=None, plates_enabled=True, mosaic_plates=False):
    """Device-resident hot path: one vd_process call over a frame batch
    (torch uint8 [n,h,w,3] on the context's GPU, or numpy). Returns (out, faces, plates)."""
    flags = _lib.VD_PROC_FACES | _lib.VD_PROC_MOSAIC
    if plates_enabled:
        flags |= _lib.VD_PROC_PLATES
        if mosaic_plates:
            flags |= _lib.VD_PROC_MOSAIC_PLATES
    return ctx.process(frames, out=out, faces=faces, plates=plates, flags=flags)
