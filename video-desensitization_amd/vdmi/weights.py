"""Weights: reference-keyed state_dicts and the VDW1 container the library loads.

The reference loads ``Retinaface_resnet50.pth`` (detect_face/face.py:52-53) and an
ultralytics ``best.pt`` (combine_detect.py:872); both are Baidu-hosted and
unavailable offline. This module therefore provides

* ``retinaface_state_dict(seed)`` / ``yolov8n_state_dict(seed, nc)``: seeded random
  weights with EXACTLY the reference's state_dict keys and shapes, so a real
  checkpoint is a drop-in replacement;
* ``load_reference_checkpoint(path)``: a converted real checkpoint
  (``torch.load(weights_only=True)``, DataParallel ``module.`` prefix stripped);
* ``pack_vdw(state_dict)``: the "VDW1" named-tensor container passed to
  ``vd_load_weights`` (magic, count, then per tensor: u16 name length, name,
  u8 dtype=0 (f32), u8 ndim, u32 dims, f32 data; little endian).

Random-weight recipe: He-normal convs; BatchNorm gamma=1, beta=0,
running_mean ~ N(0, 0.1), running_var ~ U(0.5, 1.5); two deviations keep the
activations O(1) so decoded boxes stay finite: the stem conv is scaled by 1/64
(raw-pixel input) and every bottleneck's last BN has gamma = 0.25; RetinaFace class-head bias
calibrated (tools/calibrate_weights.py) so ~40 of the 16 800 anchors score >= 0.5
on synthetic frames, which exercises threshold + NMS + mosaic at realistic counts
(tests also use stronger biases to push thousands of candidates through NMS).
"""
import struct

import numpy as np

# Calibrated by tools/calibrate_weights.py on synthetic 1920x1080 frames (seed 0):
# class-logit head scale and per-level class-1 bias giving ~0.3 % / 0.1 % / 0.1 % of the
# level-0/1/2 anchors a score >= 0.5 (~40 candidates per frame, tens of kept boxes,
# mostly small: a crowded street scene rather than one box per anchor).
CLS_HEAD_STD = 0.02
CLS_BIAS_DELTA = {0: -9.3, 1: -6.47, 2: -1.68}
# Same targets for the backbone="mobilenet" generator (tools/calibrate_weights.py --mnet).
MNET_CLS_BIAS_DELTA = {0: 0.0, 1: -4.04, 2: -2.93}
LOC_HEAD_STD = 0.01
RESIDUAL_GAMMA = 0.25


def _rng(seed):
    return np.random.default_rng(np.random.SeedSequence([0x5644, seed]))


def _conv(rng, cout, cin, k, std=None):
    fan_in = cin * k * k
    s = np.sqrt(2.0 / fan_in) if std is None else std
    return (rng.standard_normal((cout, cin, k, k)) * s).astype(np.float32)


def _bn(rng, sd, prefix, c):
    sd[prefix + ".weight"] = np.ones(c, np.float32)
    sd[prefix + ".bias"] = np.zeros(c, np.float32)
    sd[prefix + ".running_mean"] = (rng.standard_normal(c) * 0.1).astype(np.float32)
    sd[prefix + ".running_var"] = rng.uniform(0.5, 1.5, c).astype(np.float32)


def retinaface_state_dict(seed=0, cls_std=None, cls_bias=None):
    """Keys/shapes of RetinaFace(cfg_re50) (detect_face/retinaface.py:53-92 with
    torchvision resnet50 under ``body`` [ext], FPN/SSH of detect_face/nets/layers.py)."""
    rng = _rng(seed)
    sd = {}
    # stem scaled by 1/64: the input is raw pixels minus mean (rms ~75), not unit variance
    sd["body.conv1.weight"] = _conv(rng, 64, 3, 7) / np.float32(64.0)
    _bn(rng, sd, "body.bn1", 64)
    inplanes = 64
    for li, (planes, blocks, stride) in enumerate([(64, 3, 1), (128, 4, 2), (256, 6, 2), (512, 3, 2)]):
        for bi in range(blocks):
            p = f"body.layer{li + 1}.{bi}"
            sd[p + ".conv1.weight"] = _conv(rng, planes, inplanes, 1)
            _bn(rng, sd, p + ".bn1", planes)
            sd[p + ".conv2.weight"] = _conv(rng, planes, planes, 3)
            _bn(rng, sd, p + ".bn2", planes)
            sd[p + ".conv3.weight"] = _conv(rng, planes * 4, planes, 1)
            _bn(rng, sd, p + ".bn3", planes * 4)
            sd[p + ".bn3.weight"][:] = RESIDUAL_GAMMA   # keeps the residual stream O(1) over 16 blocks
            if bi == 0:
                sd[p + ".downsample.0.weight"] = _conv(rng, planes * 4, inplanes, 1)
                _bn(rng, sd, p + ".downsample.1", planes * 4)
            inplanes = planes * 4
    _fpn_ssh_heads(rng, sd, (512, 1024, 2048), 256, cls_std, cls_bias)
    return sd


def _fpn_ssh_heads(rng, sd, in_list, oc, cls_std, cls_bias):
    """FPN (layers.py:68-88), SSH x3 (:37-51) and the three head lists
    (retinaface.py:13-51) for out_channel ``oc``."""
    for i, cin in zip((1, 2, 3), in_list):
        sd[f"fpn.output{i}.0.weight"] = _conv(rng, oc, cin, 1)
        _bn(rng, sd, f"fpn.output{i}.1", oc)
    for i in (1, 2):
        sd[f"fpn.merge{i}.0.weight"] = _conv(rng, oc, oc, 3)
        _bn(rng, sd, f"fpn.merge{i}.1", oc)
    for s in (1, 2, 3):
        p = f"ssh{s}"
        q = oc // 4
        for name, cout, cin in (("conv3X3", oc // 2, oc), ("conv5X5_1", q, oc), ("conv5X5_2", q, q),
                                ("conv7X7_2", q, q), ("conv7x7_3", q, q)):
            sd[f"{p}.{name}.0.weight"] = _conv(rng, cout, cin, 3)
            _bn(rng, sd, f"{p}.{name}.1", cout)
    cstd = CLS_HEAD_STD if cls_std is None else cls_std
    cb = CLS_BIAS_DELTA if cls_bias is None else cls_bias
    for lvl in range(3):
        sd[f"ClassHead.{lvl}.conv1x1.weight"] = _conv(rng, 4, oc, 1, std=cstd)
        b = np.zeros(4, np.float32)
        b[1] = b[3] = cb[lvl] if isinstance(cb, dict) else cb   # class-1 logit of both anchors
        sd[f"ClassHead.{lvl}.conv1x1.bias"] = b
        sd[f"BboxHead.{lvl}.conv1x1.weight"] = _conv(rng, 8, oc, 1, std=LOC_HEAD_STD)
        sd[f"BboxHead.{lvl}.conv1x1.bias"] = np.zeros(8, np.float32)
        sd[f"LandmarkHead.{lvl}.conv1x1.weight"] = _conv(rng, 20, oc, 1, std=LOC_HEAD_STD)
        sd[f"LandmarkHead.{lvl}.conv1x1.bias"] = np.zeros(20, np.float32)


def retinaface_mnet_state_dict(seed=0, cls_std=None, cls_bias=None):
    """Keys/shapes of RetinaFace(cfg_mnet): MobileNetV1-0.25 under ``body``
    (detect_face/nets/mobilenet025.py:21-48, stage1/2/3 returned; the fc head is
    dropped like IntermediateLayerGetter does), FPN [64, 128, 256] -> 64, SSH(64, 64),
    heads on 64 channels (retinaface.py:60-92). Same recipe as the ResNet one
    (stem / 64 for raw-pixel input), class bias calibrated to the same pass rates."""
    rng = _rng(500 + seed)
    sd = {"body.stage1.0.0.weight": _conv(rng, 8, 3, 3) / np.float32(64.0)}
    _bn(rng, sd, "body.stage1.0.1", 8)
    chans = {1: [(8, 16), (16, 32), (32, 32), (32, 64), (64, 64)],
             2: [(64, 128)] + [(128, 128)] * 5,
             3: [(128, 256), (256, 256)]}
    for st, mods in chans.items():
        for i, (cin, cout) in enumerate(mods):
            p = f"body.stage{st}.{i + (1 if st == 1 else 0)}"
            sd[p + ".0.weight"] = _conv(rng, cin, 1, 3)   # depthwise: fan_in 9
            _bn(rng, sd, p + ".1", cin)
            sd[p + ".3.weight"] = _conv(rng, cout, cin, 1)
            _bn(rng, sd, p + ".4", cout)
    _fpn_ssh_heads(rng, sd, (64, 128, 256), 64, cls_std, MNET_CLS_BIAS_DELTA if cls_bias is None else cls_bias)
    return sd


# ----------------------------------------------------------------------------
# YOLOv8n (ultralytics yolov8.yaml, scale n = depth 0.33 / width 0.25) [ext]
# ----------------------------------------------------------------------------
def _yconv(rng, sd, p, cin, cout, k):
    sd[p + ".conv.weight"] = _conv(rng, cout, cin, k)
    _bn(rng, sd, p + ".bn", cout)


def _c2f(rng, sd, p, cin, cout, n, shortcut):
    c = cout // 2
    _yconv(rng, sd, p + ".cv1", cin, 2 * c, 1)
    _yconv(rng, sd, p + ".cv2", (2 + n) * c, cout, 1)
    for i in range(n):
        _yconv(rng, sd, f"{p}.m.{i}.cv1", c, c, 3)
        _yconv(rng, sd, f"{p}.m.{i}.cv2", c, c, 3)


YOLO_CH = {"P3": 64, "P4": 128, "P5": 256}


def yolov8n_state_dict(seed=0, nc=1, cls_bias=-0.83):
    """Keys/shapes of an ultralytics YOLOv8n DetectionModel (``model.<i>...``)."""
    rng = _rng(1000 + seed)
    sd = {}
    _yconv(rng, sd, "model.0", 3, 16, 3)
    _yconv(rng, sd, "model.1", 16, 32, 3)
    _c2f(rng, sd, "model.2", 32, 32, 1, True)
    _yconv(rng, sd, "model.3", 32, 64, 3)
    _c2f(rng, sd, "model.4", 64, 64, 2, True)
    _yconv(rng, sd, "model.5", 64, 128, 3)
    _c2f(rng, sd, "model.6", 128, 128, 2, True)
    _yconv(rng, sd, "model.7", 128, 256, 3)
    _c2f(rng, sd, "model.8", 256, 256, 1, True)
    _yconv(rng, sd, "model.9.cv1", 256, 128, 1)        # SPPF
    _yconv(rng, sd, "model.9.cv2", 512, 256, 1)
    _c2f(rng, sd, "model.12", 384, 128, 1, False)
    _c2f(rng, sd, "model.15", 192, 64, 1, False)
    _yconv(rng, sd, "model.16", 64, 64, 3)
    _c2f(rng, sd, "model.18", 192, 128, 1, False)
    _yconv(rng, sd, "model.19", 128, 128, 3)
    _c2f(rng, sd, "model.21", 384, 256, 1, False)
    c2, c3 = 64, max(64, min(nc, 100))
    for i, ch in enumerate((64, 128, 256)):
        _yconv(rng, sd, f"model.22.cv2.{i}.0", ch, c2, 3)
        _yconv(rng, sd, f"model.22.cv2.{i}.1", c2, c2, 3)
        sd[f"model.22.cv2.{i}.2.weight"] = _conv(rng, 64, c2, 1, std=0.05)
        # DFL bins biased toward short distances: plate-sized boxes rather than frame-sized
        sd[f"model.22.cv2.{i}.2.bias"] = np.tile(3.0 - 0.5 * np.arange(16), 4).astype(np.float32)
        _yconv(rng, sd, f"model.22.cv3.{i}.0", ch, c3, 3)
        _yconv(rng, sd, f"model.22.cv3.{i}.1", c3, c3, 3)
        # class std/bias calibrated on synthetic 1080p frames: ~0.1 % of anchors > 0.5
        sd[f"model.22.cv3.{i}.2.weight"] = _conv(rng, nc, c3, 1, std=1.0)
        sd[f"model.22.cv3.{i}.2.bias"] = np.full(nc, cls_bias, np.float32)
    sd["model.22.dfl.conv.weight"] = np.arange(16, dtype=np.float32).reshape(1, 16, 1, 1)
    return sd


# ----------------------------------------------------------------------------
# container + reference checkpoints
# ----------------------------------------------------------------------------
def pack_vdw(state_dict):
    """Serialise {name: float array} into the VDW1 container (integer buffers such
    as ``num_batches_tracked`` are skipped)."""
    items = []
    for k, v in state_dict.items():
        a = np.asarray(v)
        if not np.issubdtype(a.dtype, np.floating):
            continue
        items.append((k, np.ascontiguousarray(a, dtype="<f4")))
    out = [b"VDW1", struct.pack("<I", len(items))]
    for k, a in items:
        kb = k.encode()
        out.append(struct.pack("<H", len(kb)))
        out.append(kb)
        out.append(struct.pack("<BB", 0, a.ndim))
        out.append(struct.pack(f"<{a.ndim}I", *a.shape))
        out.append(a.tobytes())
    return b"".join(out)


def unpack_vdw(blob):
    mv = memoryview(blob)
    assert bytes(mv[:4]) == b"VDW1"
    (n,) = struct.unpack_from("<I", mv, 4)
    off = 8
    sd = {}
    for _ in range(n):
        (nl,) = struct.unpack_from("<H", mv, off)
        off += 2
        name = bytes(mv[off:off + nl]).decode()
        off += nl
        _, nd = struct.unpack_from("<BB", mv, off)
        off += 2
        shape = struct.unpack_from(f"<{nd}I", mv, off)
        off += 4 * nd
        cnt = int(np.prod(shape)) if nd else 1
        sd[name] = np.frombuffer(mv[off:off + 4 * cnt], "<f4").reshape(shape).copy()
        off += 4 * cnt
    return sd


def load_reference_checkpoint(path):
    """A RetinaFace .pth state_dict as saved by the reference's training code
    (weights only; never unpickles arbitrary objects)."""
    import torch
    sd = torch.load(path, map_location="cpu", weights_only=True)
    if "state_dict" in sd and isinstance(sd["state_dict"], dict):
        sd = sd["state_dict"]
    out = {}
    for k, v in sd.items():
        if k.startswith("module."):
            k = k[7:]
        out[k] = v.detach().cpu().numpy()
    return out
