"""Python handle over one libvdmi context (one GPU, one stream).

Frames may be numpy uint8 [n,h,w,3] (host) or torch uint8 tensors on the
context's GPU (device); torch is used only to hand over device pointers and
streams (plumbing), never for compute.
"""
import ctypes

import numpy as np

from . import _lib
from ._lib import check, ptr


def _is_torch(x):
    return type(x).__module__.startswith("torch")


def _frames_arg(frames):
    """-> (pointer, n, h, w, pitch, where, keepalive)."""
    if _is_torch(frames):
        if frames.dtype.__str__() != "torch.uint8" or frames.dim() != 4 or frames.shape[3] != 3:
            raise ValueError("frames must be uint8 [n,h,w,3]")
        if not frames.is_contiguous():
            frames = frames.contiguous()
        n, h, w, _ = frames.shape
        where = _lib.VD_DEVICE if frames.is_cuda else _lib.VD_HOST
        return frames.data_ptr(), n, h, w, w * 3, where, frames
    a = np.ascontiguousarray(frames, dtype=np.uint8)
    if a.ndim == 3:
        a = a[None]
    if a.ndim != 4 or a.shape[3] != 3:
        raise ValueError("frames must be uint8 [n,h,w,3]")
    n, h, w, _ = a.shape
    return a.ctypes.data, n, h, w, w * 3, _lib.VD_HOST, a


def jpeg_info(data):
    """(h, w, components) of a baseline JPEG (host-only parse, no GPU). A bytes object is
    parsed in place (its own buffer: no copy -- a 2.4-MB frame copied under the GIL for every
    frame of a batch stalled the decode / process / encode threads of GpuJpegStages)."""
    lib = _lib.load()
    h, w, c = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    if isinstance(data, bytes):
        keep = ctypes.c_char_p(data)
        buf = ctypes.cast(keep, ctypes.c_void_p)
    else:
        buf = keep = ctypes.create_string_buffer(bytes(data), len(data))
    check(lib.vd_jpeg_info(buf, len(data), ctypes.byref(h), ctypes.byref(w), ctypes.byref(c)))
    del keep
    return h.value, w.value, c.value


class DeviceBoxes:
    """vd_boxes backed by torch device tensors (kernels write them directly)."""

    def __init__(self, n, cap, device):
        import torch
        self.n, self.cap = n, cap
        self.count = torch.zeros(n, dtype=torch.int32, device=device)
        self.xyxy = torch.zeros((n, cap, 4), dtype=torch.int32, device=device)
        self.xyxy_f = torch.zeros((n, cap, 4), dtype=torch.float32, device=device)
        self.score = torch.zeros((n, cap), dtype=torch.float32, device=device)
        self.label = torch.zeros((n, cap), dtype=torch.int32, device=device)

    def struct(self):
        return _lib.vd_boxes(self.cap, _lib.VD_DEVICE, self.count.data_ptr(), self.xyxy.data_ptr(),
                             self.xyxy_f.data_ptr(), self.score.data_ptr(), self.label.data_ptr())

    def view(self, start, n):
        """Frames [start, start + n) as a DeviceBoxes sharing this one's storage (a call
        writing it fills exactly those rows)."""
        if start < 0 or n < 0 or start + n > self.n:
            raise ValueError(f"rows [{start}, {start + n}) outside [0, {self.n})")
        v = DeviceBoxes.__new__(DeviceBoxes)
        v.n, v.cap = n, self.cap
        for k in ("count", "xyxy", "xyxy_f", "score", "label"):
            setattr(v, k, getattr(self, k)[start:start + n])
        return v


class Context:
    """vd_create/vd_destroy with the reference-facing knobs as keyword args."""

    def __init__(self, device=0, precision="bf16", max_batch=64, input_shape=(640, 640), confidence=0.5,
                 nms_iou=0.4, max_boxes=256, mosaic_level=8, plate_nc=1, plate_conf=0.5, plate_iou=0.7,
                 plate_max_det=300, plate_imgsz=640, microbatch=0, microbatch_stage=2, options=None):
        lib = _lib.load()
        cfg = _lib.default_cfg()
        cfg.input_h, cfg.input_w = int(input_shape[0]), int(input_shape[1])
        cfg.max_batch = int(max_batch)
        if precision in ("fp32", "f32", "float32"):
            cfg.precision = _lib.VD_PREC_FP32
        elif precision in ("fp16", "f16", "float16", "half"):
            cfg.precision = _lib.VD_PREC_FP16
        elif precision in ("bf16", "bfloat16"):
            cfg.precision = _lib.VD_PREC_BF16
        else:
            raise ValueError(f"precision {precision!r}: expected 'bf16', 'fp16' or 'fp32'")
        cfg.confidence = float(confidence)
        cfg.nms_iou = float(nms_iou)
        cfg.max_boxes = int(max_boxes)
        cfg.mosaic_level = int(mosaic_level)
        cfg.plate_nc, cfg.plate_conf, cfg.plate_iou = int(plate_nc), float(plate_conf), float(plate_iou)
        cfg.plate_max_det, cfg.plate_imgsz = int(plate_max_det), int(plate_imgsz)
        # depth-first micro-batching of the backbone through layer<stage> (reserved[0..1])
        cfg.reserved[0], cfg.reserved[1] = int(microbatch), int(microbatch_stage)
        self.cfg = cfg
        self.device = int(device)
        self.precision = {_lib.VD_PREC_FP32: "fp32", _lib.VD_PREC_FP16: "fp16"}.get(cfg.precision, "bf16")
        h = ctypes.c_void_p()
        check(lib.vd_create(ctypes.byref(cfg), self.device, ctypes.byref(h)))
        self._h = h
        self._lib = lib
        for k, v in dict(options or {}).items():   # kernel-selection switches (vd_set_option)
            self.set_option(k, v)

    # -- lifecycle -------------------------------------------------------
    def close(self):
        if getattr(self, "_h", None) and self._h.value:
            self._lib.vd_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    def load_weights(self, net, state_dict_or_blob):
        from .weights import pack_vdw
        blob = state_dict_or_blob if isinstance(state_dict_or_blob, (bytes, bytearray)) else pack_vdw(state_dict_or_blob)
        buf = ctypes.create_string_buffer(bytes(blob), len(blob))
        check(self._lib.vd_load_weights(self._h, net, buf, len(blob), _lib.VD_WEIGHTS_VDW1))

    def set_option(self, name, value):
        check(self._lib.vd_set_option(self._h, str(name).encode(), int(value)))

    def set_debug(self, name, value):
        """Timing-only experiment switches (vdt_set_debug: "x6_dbg", "block32_dbg"); the
        results are WRONG while they are set. Never a production knob."""
        check(self._lib.vdt_set_debug(self._h, str(name).encode(), int(value)))

    def set_stream(self, stream_ptr):
        check(self._lib.vd_set_stream(self._h, stream_ptr))

    def stream(self):
        return self._lib.vd_get_stream(self._h)

    def stream_wait_event(self, event):
        """Queue a wait for a torch.cuda.Event on this context's stream (orders its next
        launches behind work recorded on another context's or torch's stream)."""
        import torch
        torch.cuda.ExternalStream(self.stream(), device=torch.device(f"cuda:{self.device}")).wait_event(event)

    def sync(self):
        check(self._lib.vd_sync(self._h))

    # -- hot path ----------------------------------------------------------
    def _boxes(self, boxes, n):
        if boxes is None:
            boxes = _lib.HostBoxes(n, self.cfg.max_boxes)
        return boxes

    def read_boxes(self, net, n, cap=None):
        """The complete keep lists of the last call for frames [0, n) (vd_read_boxes) as
        HostBoxes; cap defaults to the largest count."""
        if cap is None:
            cnt = _lib.HostBoxes(n, 1)
            check(self._lib.vd_read_boxes(self._h, net, n, ctypes.byref(cnt.struct())))
            cap = max(1, int(cnt.count.max()))
        boxes = _lib.HostBoxes(n, cap)
        check(self._lib.vd_read_boxes(self._h, net, n, ctypes.byref(boxes.struct())))
        return boxes

    def _complete(self, boxes, net, auto):
        """Library-allocated host lists never come back truncated: a frame that kept
        more than cfg.max_boxes boxes triggers a re-read of the complete lists."""
        if auto and isinstance(boxes, _lib.HostBoxes) and boxes.n and int(boxes.count.max()) > boxes.cap:
            return self.read_boxes(net, boxes.n, int(boxes.count.max()))
        return boxes

    def detect(self, frames, boxes=None):
        p, n, h, w, pitch, where, keep = _frames_arg(frames)
        auto = boxes is None
        boxes = self._boxes(boxes, n)
        s = boxes.struct()
        check(self._lib.vd_detect(self._h, p, n, h, w, pitch, where, ctypes.byref(s)))
        return self._complete(boxes, _lib.VD_NET_RETINAFACE, auto)

    def detect_plates(self, frames, boxes=None):
        p, n, h, w, pitch, where, keep = _frames_arg(frames)
        auto = boxes is None
        boxes = self._boxes(boxes, n)
        s = boxes.struct()
        check(self._lib.vd_detect_plates(self._h, p, n, h, w, pitch, where, ctypes.byref(s)))
        return self._complete(boxes, _lib.VD_NET_YOLOV8N, auto)

    def mosaic(self, frames, boxes_xyxy, counts=None, level=None, out=None):
        """Out-of-place mosaic. boxes_xyxy: int32 [n][cap][4] (host numpy) or a
        HostBoxes/DeviceBoxes; counts: int32 [n] (host) when boxes_xyxy is an array."""
        p, n, h, w, pitch, where, keep = _frames_arg(frames)
        if isinstance(boxes_xyxy, (_lib.HostBoxes, DeviceBoxes)):
            s = boxes_xyxy.struct()
        else:
            xy = np.ascontiguousarray(boxes_xyxy, np.int32).reshape(n, -1, 4)
            cnt = np.ascontiguousarray(counts if counts is not None else np.full(n, xy.shape[1]), np.int32)
            cap = max(1, xy.shape[1])
            if xy.shape[1] == 0:
                xy = np.zeros((n, 1, 4), np.int32)
            keep = (keep, xy, cnt)
            s = _lib.vd_boxes(cap, _lib.VD_HOST, ptr(cnt), ptr(xy), None, None, None)
        if out is None:
            if where == _lib.VD_HOST:
                out = np.empty((n, h, w, 3), np.uint8)
            else:
                import torch
                out = torch.empty_like(frames)
        optr = out.data_ptr() if _is_torch(out) else ptr(out)
        check(self._lib.vd_mosaic(self._h, p, optr, n, h, w, pitch, where, ctypes.byref(s),
                                  int(level or self.cfg.mosaic_level), _lib.VD_MOSAIC_OUT_OF_PLACE))
        return out

    def process(self, frames, out=None, faces=None, plates=None, flags=None):
        p, n, h, w, pitch, where, keep = _frames_arg(frames)
        if flags is None:
            flags = _lib.VD_PROC_FACES | _lib.VD_PROC_MOSAIC
        if out is None and flags & _lib.VD_PROC_MOSAIC:
            if where == _lib.VD_HOST:
                out = np.empty((n, h, w, 3), np.uint8)
            else:
                import torch
                out = torch.empty_like(frames)
        fs = ps = None
        auto_f, auto_p = faces is None, plates is None
        if flags & _lib.VD_PROC_FACES:
            faces = self._boxes(faces, n)
            fs = faces.struct()
        if flags & _lib.VD_PROC_PLATES:
            plates = self._boxes(plates, n)
            ps = plates.struct()
        optr = None if out is None else (out.data_ptr() if _is_torch(out) else ptr(out))
        check(self._lib.vd_process(self._h, p, optr, n, h, w, pitch, where, flags,
                                   ctypes.byref(fs) if fs is not None else None,
                                   ctypes.byref(ps) if ps is not None else None))
        if flags & _lib.VD_PROC_FACES:
            faces = self._complete(faces, _lib.VD_NET_RETINAFACE, auto_f)
        if flags & _lib.VD_PROC_PLATES:
            plates = self._complete(plates, _lib.VD_NET_YOLOV8N, auto_p)
        return out, faces, plates

    # -- frame I/O ------------------------------------------------------------
    def jpeg_decode(self, jpegs, out=None):
        """Baseline JPEG frames (a list of bytes, all one size and layout) -> RGB
        uint8 [n,h,w,3], bit-identical to libjpeg-turbo's default decode (what
        cv2.imread + BGR->RGB gives the reference, combine_detect.py:167-172).
        `out`: a torch uint8 device tensor (decoded in place on the GPU, queued on
        the context stream -- ready to pass to process()) or None (numpy result)."""
        jpegs = [bytes(j) for j in jpegs]
        n = len(jpegs)
        if n == 0:
            raise ValueError("no frames")
        h, w, _ = jpeg_info(jpegs[0])
        # the bytes objects' own buffers (immutable; the library only reads them): no copy
        bufs = [ctypes.c_char_p(j) for j in jpegs]
        ptrs = (ctypes.c_void_p * n)(*[ctypes.cast(b, ctypes.c_void_p).value for b in bufs])
        sizes = (ctypes.c_size_t * n)(*[len(j) for j in jpegs])
        if out is None:
            out = np.empty((n, h, w, 3), np.uint8)
        if _is_torch(out):
            if tuple(out.shape) != (n, h, w, 3) or not out.is_contiguous():
                raise ValueError(f"out must be contiguous uint8 [{n},{h},{w},3]")
            where, optr = (_lib.VD_DEVICE if out.is_cuda else _lib.VD_HOST), out.data_ptr()
        else:
            if out.shape != (n, h, w, 3) or out.dtype != np.uint8 or not out.flags["C_CONTIGUOUS"]:
                raise ValueError(f"out must be C-contiguous uint8 [{n},{h},{w},3]")
            where, optr = _lib.VD_HOST, ptr(out)
        check(self._lib.vd_jpeg_decode(self._h, ptrs, sizes, n, optr, h, w, w * 3, where))
        return out

    def jdec_passes(self):
        """Synchronisation passes of the last jpeg_decode's device entropy stage (pass 0
        included; 0 when the host entropy stage ran) -- test / bench hook."""
        p = ctypes.c_int(0)
        check(self._lib.vdt_jdec_stats(self._h, ctypes.byref(p)))
        return p.value

    def jpeg_encode(self, frames, quality=95, subsampling=2, copy=True):
        """RGB uint8 frames [n,h,w,3] (numpy, or a torch tensor on the GPU: encoded
        from device memory, no D2H of pixels) -> list of JFIF bytes, bit-identical to
        libjpeg-turbo's compressor (Pillow ``Image.save(..., quality=quality,
        subsampling=subsampling)``; cv2.imwrite's defaults are quality 95, 4:2:0 --
        the reference's frame write, combine_detect.py:174-180).
        copy=False: read-only memoryviews into one buffer of this call (no per-frame
        copy into bytes objects; the buffer lives as long as any view does).
        """
        p, n, h, w, pitch, where, keep = _frames_arg(frames)
        sizes = (ctypes.c_size_t * n)()
        # typical frames need < 3 B/pixel; on VD_ERR_CAPACITY the device coder reports
        # each frame's bound in sizes[] (the host coder 0: then the bound of any
        # baseline block, 63 AC codes of 26 bits + DC, every byte stuffed)
        caps = [h * w * 3 + 65536]
        while len(caps) < 3:
            cap = caps[-1]
            if copy:   # one staging buffer per context, reused (fresh pages would fault in on every call)
                out = getattr(self, "_jenc_buf", None)
                if out is None or out.size < n * cap:
                    out = self._jenc_buf = np.empty(n * cap, np.uint8)
            else:      # this call's own buffer: the views stay valid (first touch on the copy threads)
                out = np.empty(n * cap, np.uint8)
            rc = self._lib.vd_jpeg_encode(self._h, p, n, h, w, pitch, where, int(quality), int(subsampling),
                                          ptr(out), cap, sizes)
            if rc != _lib.VD_ERR_CAPACITY:
                break
            need = max(sizes[i] for i in range(n))
            caps.append(need + 64 if need > cap else h * w * 20 + 65536)
        check(rc)
        del keep
        if not copy:
            mv = memoryview(out).toreadonly()
            return [mv[i * cap:i * cap + sizes[i]] for i in range(n)]
        return [out[i * cap:i * cap + sizes[i]].tobytes() for i in range(n)]

    # -- instrumentation ------------------------------------------------------
    def timing(self, on=True):
        check(self._lib.vd_timing_enable(self._h, 1 if on else 0))

    def timing_reset(self):
        check(self._lib.vd_timing_reset(self._h))

    def timing_read(self, fam):
        ms, n, work = ctypes.c_double(), ctypes.c_int64(), ctypes.c_double()
        check(self._lib.vd_timing_read(self._h, fam, ctypes.byref(ms), ctypes.byref(n), ctypes.byref(work)))
        return ms.value, n.value, work.value

    # -- test hooks --------------------------------------------------------------
    def letterbox(self, frames, cpad=4):
        p, n, h, w, pitch, where, keep = _frames_arg(frames)
        out = np.zeros((n, self.cfg.input_h, self.cfg.input_w, cpad), np.float32)
        check(self._lib.vdt_letterbox(self._h, p, n, h, w, pitch, where, ptr(out), cpad))
        return out

    def forward_heads(self, frames):
        p, n, h, w, pitch, where, keep = _frames_arg(frames)
        A = sum((self.cfg.input_h // s) * (self.cfg.input_w // s) * 2 for s in (8, 16, 32))
        loc = np.zeros((n, A, 4), np.float32)
        conf = np.zeros((n, A, 2), np.float32)
        landm = np.zeros((n, A, 10), np.float32)
        check(self._lib.vdt_forward_heads(self._h, p, n, h, w, pitch, where, ptr(loc), ptr(conf), ptr(landm)))
        return loc, conf, landm

    def postprocess(self, loc, conf, img_hw, cap=None):
        loc = np.ascontiguousarray(loc, np.float32)
        conf = np.ascontiguousarray(conf, np.float32)
        n = loc.shape[0]
        hw = np.ascontiguousarray(np.broadcast_to(np.asarray(img_hw, np.int32), (n, 2)))
        boxes = _lib.HostBoxes(n, cap or self.cfg.max_boxes)
        s = boxes.struct()
        check(self._lib.vdt_postprocess(self._h, ptr(loc), ptr(conf), n, ptr(hw), ctypes.byref(s)))
        return self._complete(boxes, _lib.VD_NET_RETINAFACE, cap is None)

    def plate_raw(self, frames):
        """Raw YOLO head outputs [n][64+nc][A] (DFL logits | class logits), f32."""
        p, n, h, w, pitch, where, keep = _frames_arg(frames)
        A = ctypes.c_int()
        check(self._lib.vdt_plate_raw(self._h, p, n, h, w, pitch, where, None, ctypes.byref(A)))
        out = np.zeros((n, 64 + self.cfg.plate_nc, A.value), np.float32)
        check(self._lib.vdt_plate_raw(self._h, p, n, h, w, pitch, where, ptr(out), ctypes.byref(A)))
        return out

    def bottleneck(self, x, w1, bn1, w2, bn2, w3, bn3, wd=None, bnd=None, fused=True):
        """One ResNet layer1 bottleneck (bf16 or fp32 context): x f32 NHWC [n,h,w,cin] -> f32
        NHWC [n,h,w,256]; bnK = concat(scale, shift). fused: the one-kernel block
        (block.hip / block32.hip), else the conv-by-conv chain."""
        f = lambda a: None if a is None else np.ascontiguousarray(a, np.float32)
        x = f(x)
        n, h, wd_, cin = x.shape
        y = np.zeros((n, h, wd_, 256), np.float32)
        args = [f(a) for a in (w1, bn1, w2, bn2, w3, bn3, wd, bnd)]
        check(self._lib.vdt_bottleneck(self._h, ptr(x), n, h, wd_, cin, *[ptr(a) for a in args], int(bool(fused)),
                                       ptr(y)))
        return y

    def conv2d(self, x, w, stride=1, pad=0, scale=None, shift=None, act=0, slope=0.0, res=None, res_mode=0):
        """x: f32 NHWC [n,h,w,cin]; w: f32 [cout,cin,kh,kw] -> f32 NHWC."""
        x = np.ascontiguousarray(x, np.float32)
        w = np.ascontiguousarray(w, np.float32)
        n, h, wd, cin = x.shape
        cout, _, kh, kw = w.shape
        scale = np.ascontiguousarray(np.ones(cout, np.float32) if scale is None else scale, np.float32)
        shift = np.ascontiguousarray(np.zeros(cout, np.float32) if shift is None else shift, np.float32)
        oh, ow = (h + 2 * pad - kh) // stride + 1, (wd + 2 * pad - kw) // stride + 1
        y = np.zeros((n, oh, ow, cout), np.float32)
        r = None if res is None else np.ascontiguousarray(res, np.float32)
        o1, o2 = ctypes.c_int(), ctypes.c_int()
        check(self._lib.vdt_conv2d(self._h, ptr(x), n, h, wd, cin, ptr(w), cout, kh, kw, stride, pad, ptr(scale),
                                   ptr(shift), act, float(slope), ptr(r), res_mode, ptr(y), ctypes.byref(o1),
                                   ctypes.byref(o2)))
        return y
