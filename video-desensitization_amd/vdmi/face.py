"""Drop-in ``Retinaface`` (detect_face/face.py:14-150) backed by libvdmi.

Same constructor keywords and defaults (face.py:15-23), same ``.device``
attribute (read at combine_detect.py:866), same ``detect_images`` contract
(face.py:120-150): a list of uint8 HxWx3 RGB arrays in, a list of
``(image, [[x1, y1, x2, y2], ...])`` out, boxes as Python floats in source
pixels, in NMS (descending score) order. Everything between — letterbox,
ResNet-50 (or MobileNet-0.25)/FPN/SSH forward, decode, NMS, correction — runs in HIP kernels.

Differences, all deliberate:
* ``cuda=False`` raises: the product path has no CPU fallback (the reference's
  own CPU path crashes in retinaface_correct_boxes' ``.cuda()``, utils_bbox.py:118).
* ``model_path`` missing on disk raises FileNotFoundError (a desensitisation run
  on random weights would leave every face visible while appearing to succeed).
  Seeded random weights with the reference keys are an explicit opt-in,
  ``weights="random"`` (tests, benchmarks).
* The returned image is the caller's array itself, not a copy (face.py:129 copies;
  the driver never reads it, combine_detect.py:237).
* Extra keywords: ``precision`` ("fp32" default: f32 activations and weights, each
  conv on scaled fp16 pairs -- three f16 MFMA products, f32 accumulation, heads
  within 6e-6 of the torch-CPU fp32 forward; option ``f32_split=0`` runs exact-f32
  MFMA instead; "bf16" / "fp16" trade box parity for 2-3x throughput, see
  INTEGRATION.md), ``max_batch``, ``device_ids`` / ``device_index``, ``seed``,
  ``weights`` (a state_dict, or "random"), ``options`` (kernel-selection switches).
* Devices (face.py:55-56 wraps the net in ``nn.DataParallel``: every forward is
  split over ALL visible GPUs, the weights re-broadcast each time): one context per
  device, weights uploaded once each; ``detect_images`` cuts the image list into
  contiguous shards, one per device, each driven by its own host thread (the C
  calls release the GIL). Default devices: ``device_ids`` if given ("all" = every
  visible GPU), else ``[device_index]`` if given, else ``[LOCAL_RANK]`` inside a
  torchrun rank (one GPU per process: vdmi.dist), else every visible GPU -- what
  DataParallel uses.
"""
import os

import numpy as np

from . import _lib
from .context import Context
from .weights import load_reference_checkpoint, retinaface_mnet_state_dict, retinaface_state_dict


def resolve_devices(device_ids=None, device_index=None):
    """The GPUs a drop-in detector spreads over (see the module docstring)."""
    def visible():
        try:
            import torch
            return max(1, torch.cuda.device_count())
        except Exception:
            return 1
    if device_ids is not None:
        ids = list(range(visible())) if device_ids == "all" else [int(d) for d in device_ids]
        if not ids:
            raise ValueError("device_ids is empty")
        return ids
    if device_index is not None:
        return [int(device_index)]
    if os.environ.get("LOCAL_RANK") not in (None, ""):
        return [int(os.environ["LOCAL_RANK"])]
    return list(range(visible()))


def split_run(ctxs, items, fn):
    """fn(ctx, sub_list) -> list per item, with `items` cut into contiguous shards,
    one per context, each on its own thread; results in item order."""
    from .dist import run_on_devices, shard_range
    if len(ctxs) == 1 or len(items) <= 1:
        return fn(ctxs[0], items)
    spans = [shard_range(len(items), len(ctxs), i) for i in range(len(ctxs))]
    parts = run_on_devices(lambda i, sp: fn(ctxs[i], items[sp[0]:sp[1]]) if sp[1] > sp[0] else [], spans,
                           devices=[c.device for c in ctxs])
    return [r for p in parts for r in p]


class Retinaface(object):
    _defaults = {
        "model_path": "model_data/Retinaface_resnet50.pth",
        "backbone": "resnet50",
        "confidence": 0.5,
        "nms_iou": 0.45,
        "input_shape": [1280, 1280, 3],
        "letterbox_image": True,
        "cuda": True,
        # vdmi extras
        "precision": "fp32",
        "max_batch": 64,
        "device_index": None,
        "device_ids": None,
        "seed": 0,
        "weights": None,
        "max_boxes": 256,
    }

    @classmethod
    def get_defaults(cls, n):
        return cls._defaults.get(n, f"Unrecognized attribute name '{n}'")

    def __init__(self, **kwargs):
        self.__dict__.update(self._defaults)
        for name, value in kwargs.items():
            setattr(self, name, value)
        if self.backbone not in ("resnet50", "mobilenet"):   # face.py:35: cfg_mnet / cfg_re50
            raise ValueError(f"backbone must be 'resnet50' or 'mobilenet', got {self.backbone!r}")
        if not self.letterbox_image:
            raise ValueError("Batch inference requires letterbox_image=True for shape alignment.")  # face.py:80
        if not self.cuda:
            raise RuntimeError("vdmi.Retinaface runs on the GPU only (no CPU fallback)")
        self.device_ids = resolve_devices(self.device_ids, self.device_index)
        self.device_index = self.device_ids[0]
        try:
            import torch
            self.device = torch.device(f"cuda:{self.device_index}")
        except Exception:  # torch is optional plumbing
            self.device = f"cuda:{self.device_index}"
        self.options = getattr(self, "options", None)
        self.ctxs = [Context(device=d, precision=self.precision, max_batch=self.max_batch,
                             input_shape=self.input_shape[:2], confidence=self.confidence, nms_iou=self.nms_iou,
                             max_boxes=self.max_boxes, options=self.options) for d in self.device_ids]
        self.ctx = self.ctxs[0]
        self.generate()

    def generate(self):
        """face.py:50-60: load weights once (device-resident; no DataParallel replicate)."""
        if isinstance(self.weights, str) and self.weights == "random":   # explicit opt-in (tests, bench)
            sd = (retinaface_mnet_state_dict if self.backbone == "mobilenet" else retinaface_state_dict)(self.seed)
        elif self.weights is not None:
            sd = self.weights
        elif self.model_path and os.path.exists(self.model_path):
            sd = load_reference_checkpoint(self.model_path)
        else:
            raise FileNotFoundError(f"RetinaFace checkpoint {self.model_path!r} not found (pass model_path=, "
                                    "weights=<state_dict>, or weights='random' for seeded test weights)")
        self.state_dict = sd           # kept for a fused face+plate context (vdmi.pipeline)
        for c in self.ctxs:            # once per device (DataParallel re-broadcasts every forward)
            c.load_weights(_lib.VD_NET_RETINAFACE, sd)

    def detect_boxes(self, images):
        """Per image: (float32 boxes [M,4], int boxes [M,4], scores [M]) in NMS order;
        the list is split over the detector's devices (one thread each)."""
        if not isinstance(images, list):
            images = [images]
        return split_run(self.ctxs, images, self._detect_on)

    def _detect_on(self, ctx, images):
        out = [None] * len(images)
        groups = {}
        for i, img in enumerate(images):
            groups.setdefault(img.shape[:2], []).append(i)
        for (h, w), idx in groups.items():
            for s in range(0, len(idx), self.max_batch):
                chunk = idx[s:s + self.max_batch]
                batch = np.stack([images[i] for i in chunk]) if len(chunk) > 1 else images[chunk[0]][None]
                boxes = ctx.detect(np.ascontiguousarray(batch, np.uint8))
                for j, i in enumerate(chunk):
                    xi, xf, sc, _ = boxes.frame(j)
                    out[i] = (xf.copy(), xi.copy(), sc.copy())
        return out

    def detect_images(self, images):
        """face.py:120-150."""
        if not isinstance(images, list):
            images = [images]
        res = self.detect_boxes(images)
        return [(img, r[0].tolist()) for img, r in zip(images, res)]
