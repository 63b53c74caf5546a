"""Drop-in for the ultralytics plate detector the reference drives
(``YOLO(plate_model_path).cuda()`` at combine_detect.py:872, called as
``plate_detector(batch_images, verbose=False, conf=0.5)`` at :217 and probed with
``next(plate_detector.model.parameters()).device`` at :876).

``__call__`` returns one ``Results``-like object per image whose ``.boxes``
carries ``xyxy`` / ``conf`` / ``cls`` (numpy, source pixels, NMS order), as
ultralytics does [ext]. Note the reference never uses them: its tuple check at
combine_detect.py:239 always yields [] for Results objects. ``vdmi.pipeline``
reproduces that by default and offers the intended behaviour as an option.

Architecture: YOLOv8n. The reference's ``best.pt`` is a
pickled ultralytics object that is never unpickled here (it would execute code).
Accepted weights: a state_dict file with ``model.<i>...`` keys loadable by
``torch.load(weights_only=True)`` -- convert once where ultralytics is installed:
``torch.save(YOLO("best.pt").model.float().state_dict(), "best_sd.pt")`` -- a VDW1
file, or ``weights=<state_dict>``. A missing or unloadable file raises;
``weights="random"`` (seeded, reference keys) is an explicit opt-in for tests.
"""
import os

import numpy as np

from . import _lib
from .context import Context
from .weights import yolov8n_state_dict


class Boxes:
    def __init__(self, xyxy, conf, cls):
        self.xyxy, self.conf, self.cls = xyxy, conf, cls
        self.data = np.concatenate([xyxy, conf[:, None], cls[:, None].astype(np.float32)], 1) if len(xyxy) else \
            np.zeros((0, 6), np.float32)

    def __len__(self):
        return len(self.xyxy)


class Results:
    def __init__(self, orig_img, boxes, names):
        self.orig_img = orig_img
        self.orig_shape = orig_img.shape[:2]
        self.boxes = boxes
        self.names = names

    def __len__(self):
        return len(self.boxes)


class _ModelProxy:
    """``.parameters()`` for combine_detect.py:876."""

    def __init__(self, device):
        self._device = device

    def parameters(self):
        try:
            import torch
            yield torch.nn.Parameter(torch.empty(0, device=self._device))
        except Exception:   # torch absent: a stand-in with .device
            yield type("P", (), {"device": self._device})()


def load_plate_weights(path):
    """A YOLOv8 state_dict file (torch weights_only) or a VDW1 file -> {name: array}."""
    if not path or not os.path.exists(path):
        raise FileNotFoundError(f"plate weights {path!r} not found (pass a converted state_dict / VDW1 file, "
                                "weights=<state_dict>, or weights='random' for seeded test weights)")
    with open(path, "rb") as f:
        magic = f.read(4)
    if magic == b"VDW1":
        from .weights import unpack_vdw
        return unpack_vdw(open(path, "rb").read())
    import torch
    try:
        sd = torch.load(path, map_location="cpu", weights_only=True)
    except Exception as e:   # a pickled ultralytics model object: refused by the safe loader
        raise ValueError(f"{path}: not a weights-only state_dict (a pickled ultralytics checkpoint is never "
                         "unpickled here). Convert it where ultralytics is installed: torch.save(YOLO(path)."
                         "model.float().state_dict(), 'best_sd.pt')") from e
    if isinstance(sd, dict) and isinstance(sd.get("model"), dict):
        sd = sd["model"]
    if not isinstance(sd, dict) or not any(k.startswith("model.") for k in sd):
        raise ValueError(f"{path}: no 'model.<i>...' keys: not a YOLOv8 DetectionModel state_dict")
    return {k: v.detach().float().cpu().numpy() for k, v in sd.items() if hasattr(v, "detach")}


class YOLO:
    """ultralytics-style plate detector on libvdmi."""

    def __init__(self, model="best.pt", nc=1, weights=None, precision="fp32", max_batch=64, device_index=None,
                 seed=0, imgsz=640, iou=0.7, max_det=300, names=None, device_ids=None):
        from .face import resolve_devices
        self.nc = nc
        self.names = names or {i: f"plate{i}" if nc > 1 else "plate" for i in range(nc)}
        # devices as vdmi.Retinaface resolves them (one context each; a call's image list
        # is split over them, one thread per device)
        self.device_ids = resolve_devices(device_ids, device_index)
        self.device_index = self.device_ids[0]
        self.max_batch = max_batch
        self.ctxs = [Context(device=d, precision=precision, max_batch=max_batch, plate_nc=nc, plate_iou=iou,
                             plate_max_det=max_det, plate_imgsz=imgsz) for d in self.device_ids]
        self.ctx = self.ctxs[0]
        if isinstance(weights, str) and weights == "random":   # explicit opt-in (tests, bench)
            weights = yolov8n_state_dict(seed, nc)
        elif weights is None:
            weights = load_plate_weights(model)
        self.state_dict = weights      # kept for a fused face+plate context (vdmi.pipeline)
        for c in self.ctxs:
            c.load_weights(_lib.VD_NET_YOLOV8N, weights)
        self.model = _ModelProxy(f"cuda:{self.device_index}")
        self._conf = 0.5

    def cuda(self):
        return self

    def predict(self, source, conf=0.5, verbose=False, **_):
        return self(source, conf=conf, verbose=verbose)

    def __call__(self, source, verbose=False, conf=0.5, **_):
        from .face import split_run
        imgs = source if isinstance(source, list) else [source]
        if abs(conf - self.ctx.cfg.plate_conf) > 1e-12:
            raise ValueError(f"conf={conf} differs from the context's plate_conf={self.ctx.cfg.plate_conf}")
        return split_run(self.ctxs, imgs, self._detect_on)

    def _detect_on(self, ctx, imgs):
        out = [None] * len(imgs)
        groups = {}
        for i, im in enumerate(imgs):
            groups.setdefault(im.shape[:2], []).append(i)
        for (h, w), idx in groups.items():
            for s in range(0, len(idx), self.max_batch):
                chunk = idx[s:s + self.max_batch]
                batch = np.stack([imgs[i] for i in chunk]) if len(chunk) > 1 else imgs[chunk[0]][None]
                bx = ctx.detect_plates(np.ascontiguousarray(batch, np.uint8))
                for j, i in enumerate(chunk):
                    _, xf, sc, lab = bx.frame(j)
                    out[i] = Results(imgs[i], Boxes(xf.copy(), sc.copy(), lab.astype(np.float32)), self.names)
        return out


PlateDetector = YOLO
