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
import logging
import os
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


def fused_context(face_detector, plate_detector, batch_size):
    """One context holding both drop-ins' weights and the face detector's knobs
    (cached on the face detector)."""
    from .context import Context
    key = (id(plate_detector), int(batch_size))
    cache = getattr(face_detector, "_fused", None)
    if cache and cache[0] == key:
        return cache[1]
    fd, pd = face_detector, plate_detector
    ctx = Context(device=fd.device_index, precision=fd.precision, max_batch=max(int(batch_size), 1),
                  input_shape=fd.input_shape[:2], confidence=fd.confidence, nms_iou=fd.nms_iou,
                  max_boxes=fd.max_boxes, plate_nc=pd.nc, plate_conf=pd.ctx.cfg.plate_conf,
                  plate_iou=pd.ctx.cfg.plate_iou, plate_max_det=pd.ctx.cfg.plate_max_det,
                  plate_imgsz=pd.ctx.cfg.plate_imgsz)
    ctx.load_weights(_lib.VD_NET_RETINAFACE, fd.state_dict)
    ctx.load_weights(_lib.VD_NET_YOLOV8N, pd.state_dict)
    face_detector._fused = (key, ctx)
    return ctx


def _is_vdmi_pair(face_detector, plate_detector):
    from .face import Retinaface
    from .plate import YOLO
    return isinstance(face_detector, Retinaface) and isinstance(plate_detector, YOLO)


def batch_process_images(input_dir, output_dir, face_detector, plate_detector, batch_size=16,
                         loader=None, saver=None, mosaic_plates=False, mosaic_level=8, num_workers=6,
                         gpu_codec="auto", jpeg_quality=95):
    """combine_detect.py:183-277. Returns (total_processed, total_faces, total_plates).

    gpu_codec ("auto" | True | False): with vdmi detectors, no custom loader/saver and
    only .jpg/.jpeg frames (what the reference's ffmpeg split writes), the frames are
    read as bytes, decoded on the GPU (vd_jpeg_decode), processed and encoded on the
    GPU (vd_jpeg_encode, cv2.imwrite's quality 95 / 4:2:0), so pixels never cross
    PCIe; the bytes written equal libjpeg-turbo's encode of the processed frames."""
    logger = logging.getLogger("VideoProcessor.batch_process_images")
    custom_io = loader is not None or saver is not None
    if gpu_codec is True and custom_io:
        raise ValueError("gpu_codec=True reads and writes JPEG bytes itself: it cannot use a custom loader/saver")
    loader = loader or load_image_rgb
    saver = saver or save_output_image
    image_paths = [os.path.join(input_dir, f) for f in os.listdir(input_dir) if f.lower().endswith(IMAGE_EXT)]
    os.makedirs(output_dir, exist_ok=True)
    batches = [image_paths[i:i + batch_size] for i in range(0, len(image_paths), batch_size)]
    io = ThreadPoolExecutor(max_workers=num_workers)
    try:
        fused = _is_vdmi_pair(face_detector, plate_detector) and mosaic_level == face_detector.ctx.cfg.mosaic_level
        all_jpeg = all(p.lower().endswith((".jpg", ".jpeg")) for p in image_paths)
        if fused and gpu_codec and (gpu_codec is True or (not custom_io and all_jpeg)):
            res = _gpu_codec_batches(batches, output_dir, face_detector, plate_detector, batch_size, mosaic_plates,
                                     io, logger, jpeg_quality)
        elif fused:
            res = _fused_batches(batches, output_dir, face_detector, plate_detector, batch_size, loader, saver,
                                 mosaic_plates, io, logger)
        else:
            res = _threaded_batches(batches, output_dir, face_detector, plate_detector, loader, saver,
                                    mosaic_plates, mosaic_level, io, logger)
    finally:
        io.shutdown(wait=True)
    logger.info(f"processed {res[0]} images: {res[1]} faces, {res[2]} plates")
    return res


def _save_all(futs, logger):
    for f in futs:
        try:
            f.result()
        except Exception as e:
            logger.error(f"saving failed: {e}")


def _fused_batches(batches, output_dir, face_detector, plate_detector, batch_size, loader, saver, mosaic_plates,
                   io, logger):
    """The vdmi path, streaming: decode batch b+1 (threads) while batch b is on the
    GPU (FramePipeline: one vd_process per batch), collect batch b-1 and hand its
    frames to the encoder threads. Frames of another size get their own pipeline;
    a batch whose inference fails is dropped (combine_detect.py:226-228), a load
    failure aborts the call (:209-211)."""
    totals = [0, 0, 0]
    save_futs = []
    ctx = fused_context(face_detector, plate_detector, batch_size)
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
            pending = _submit_groups(files, imgs, pipes, ctx, batch_size, mosaic_plates, pending, finish, logger)
    finally:
        if fut is not None:
            fut.cancel()
        if pending is not None:
            finish(pending)
        for pipe in pipes.values():
            pipe.close()
        _save_all(save_futs, logger)
    return tuple(totals)


def _submit_groups(files, imgs, pipes, ctx, batch_size, mosaic_plates, pending, finish, logger):
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
            cur = (pipes[shape], pipes[shape].submit(np.stack([im for _, im in items])),
                   [f for f, _ in items])
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
                       quality):
    """Frame I/O on the GPU: file bytes (reader threads) -> vd_jpeg_decode into
    device frames -> one vd_process (faces | plates | mosaic) -> vd_jpeg_encode from
    device memory -> writer threads. Batch i+1 is read and decoded (its host Huffman
    threads and IDCT kernels, on a second weight-less context and stream) while
    batch i is processed and encoded. A frame the GPU decoder does not take
    (progressive, other layout) is decoded by the host loader; a batch whose
    inference fails is dropped (combine_detect.py:226-228)."""
    import torch
    from .context import Context, DeviceBoxes, jpeg_info
    ctx = fused_context(face_detector, plate_detector, batch_size)
    dev = torch.device(f"cuda:{ctx.device}")
    dctx = Context(device=ctx.device, precision="fp32", max_batch=max(int(batch_size), 1))
    flags = _lib.VD_PROC_FACES | _lib.VD_PROC_MOSAIC | _lib.VD_PROC_PLATES
    if mosaic_plates:
        flags |= _lib.VD_PROC_MOSAIC_PLATES
    faces = DeviceBoxes(batch_size, 256, dev)
    plates = DeviceBoxes(batch_size, 256, dev)
    totals = [0, 0, 0]
    save_futs = []

    def load(files):
        """files -> [(items, device frames)] per frame size, decoded and synchronised"""
        blobs = list(io.map(_read_bytes, files))
        groups = {}
        for f, b in zip(files, blobs):
            try:
                key = jpeg_info(b)[:2]
            except Exception:
                key = load_image_rgb(f).shape[:2]
            groups.setdefault(key, []).append((f, b))
        out = []
        for (h, w), items in groups.items():
            d_in = torch.empty((len(items), h, w, 3), dtype=torch.uint8, device=dev)
            try:
                dctx.jpeg_decode([b for _, b in items], out=d_in)
                dctx.sync()
            except Exception:                # not a layout the GPU decoder takes: host decode
                d_in.copy_(torch.from_numpy(np.stack([load_image_rgb(f) for f, _ in items])))
                torch.cuda.synchronize(dev)  # the copy ran on torch's stream, not a context's
            out.append((items, d_in))
        return out

    # batch i+1 decoded (dctx), batch i processed (ctx), batch i-1 encoded (ectx): three
    # contexts, each with its own stream and lock, so the three stages overlap
    ectx = Context(device=ctx.device, precision="fp32", max_batch=max(int(batch_size), 1))

    def encode(items, out):
        jpgs = ectx.jpeg_encode(out, quality=quality, subsampling=2, copy=False)
        return [io.submit(_write_bytes, data, os.path.join(output_dir, f"processed_{os.path.basename(path)}"))
                for (path, _), data in zip(items, jpgs)]

    def collect(fut):
        try:
            save_futs.extend(fut.result())
        except Exception as e:           # combine_detect.py:226-228: the batch is dropped
            logger.error(f"parallel inference failed: {e}")
            return False
        return True

    ahead, behind = ThreadPoolExecutor(1), ThreadPoolExecutor(1)
    enc = []                             # (future, counts) of batches being encoded
    try:
        fut = ahead.submit(load, batches[0]) if batches else None
        for bi in range(len(batches)):
            decoded = fut.result()       # a load failure propagates (combine_detect.py:209-211)
            fut = ahead.submit(load, batches[bi + 1]) if bi + 1 < len(batches) else None
            for items, d_in in decoded:
                try:
                    out, fc, pc = ctx.process(d_in, faces=faces, plates=plates, flags=flags)
                    ctx.sync()           # the encode context reads `out` on its own stream
                except Exception as e:   # combine_detect.py:226-228: the batch is dropped
                    logger.error(f"parallel inference failed: {e}")
                    continue
                n = len(items)
                counts = (n, int(fc.count[:n].sum().item()), int(pc.count[:n].sum().item()) if mosaic_plates else 0)
                enc.append((behind.submit(encode, items, out), counts))
                while len(enc) > 1:      # at most one batch encoding behind the one just processed
                    f0, c0 = enc.pop(0)
                    if collect(f0):
                        totals[0] += c0[0]; totals[1] += c0[1]; totals[2] += c0[2]
    finally:
        # every batch already handed to the encoder is finished (its errors logged, its
        # writes queued) before the saves are waited on -- also when a load failure aborts
        while enc:
            f0, c0 = enc.pop(0)
            if collect(f0):
                totals[0] += c0[0]; totals[1] += c0[1]; totals[2] += c0[2]
        ahead.shutdown()
        behind.shutdown()
        dctx.close()
        ectx.close()
        _save_all(save_futs, logger)
    return tuple(totals)


def _threaded_batches(batches, output_dir, face_detector, plate_detector, loader, saver, mosaic_plates,
                      mosaic_level, io, logger):
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
        for j in range(len(batch_images)):
            face_boxes = _boxes_of(face_results[j])
            if mosaic_plates and not isinstance(plate_results[j], tuple):
                plate_boxes = plate_results[j].boxes.xyxy.tolist()
            else:
                plate_boxes = _boxes_of(plate_results[j])
            boxes = [(int(x1), int(y1), int(x2), int(y2)) for x1, y1, x2, y2 in face_boxes]
            boxes += [(int(x1), int(y1), int(x2), int(y2)) for x1, y1, x2, y2 in plate_boxes]
            per_frame.append(boxes)
            faces += len(face_boxes)
            plates += len(plate_boxes)
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
