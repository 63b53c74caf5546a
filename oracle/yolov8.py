"""YOLOv8n plate detector on torch-CPU fp32 + ultralytics post-processing in
numpy — TEST INFRASTRUCTURE ONLY. PARITY UNPINNED: ultralytics is absent from
the reference tree and from this container and its version is unpinned by the
reference (README.md:16, FLPR.dockerfile:55; a commented ultralytics==8.0.49 at
requirements.txt:81), so this restates the published upstream algorithm:

* model: yolov8.yaml at scale n (depth 0.33, width 0.25) — Conv(k, s, autopad)
  + BatchNorm(eps 1e-3) + SiLU, C2f(n, shortcut), SPPF(k=5), nearest Upsample,
  Concat, Detect(reg_max 16, c2 = c3 = 64, DFL), state_dict keys ``model.<i>...``;
* predict (combine_detect.py:217): LetterBox(640, auto, stride 32, pad 114),
  BGR<->RGB flip, /255 (oracle/letterbox.py); Detect inference (DFL softmax
  expectation, dist2bbox xywh * stride, class sigmoid); non_max_suppression
  (candidates max class score > conf, xywh2xyxy, class offset 7680, torchvision
  nms at IoU 0.7, max_det 300); scale_boxes (gain, rounded pad, clip).
The plate boxes never reach the reference's mosaic (combine_detect.py:239), so
the reference's pixel output does not depend on any of this.
"""
import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from .bbox import nms_torchvision
from .vdexp import vd_expf

F32 = np.float32


class Conv(nn.Module):
    def __init__(self, c1, c2, k=1, s=1):
        super().__init__()
        self.conv = nn.Conv2d(c1, c2, k, s, k // 2, bias=False)
        self.bn = nn.BatchNorm2d(c2, eps=1e-3)

    def forward(self, x):
        return F.silu(self.bn(self.conv(x)))


class Bottleneck(nn.Module):
    def __init__(self, c1, c2, shortcut=True):
        super().__init__()
        self.cv1 = Conv(c1, c2, 3)
        self.cv2 = Conv(c2, c2, 3)
        self.add = shortcut and c1 == c2

    def forward(self, x):
        return x + self.cv2(self.cv1(x)) if self.add else self.cv2(self.cv1(x))


class C2f(nn.Module):
    def __init__(self, c1, c2, n=1, shortcut=False):
        super().__init__()
        self.c = c2 // 2
        self.cv1 = Conv(c1, 2 * self.c, 1)
        self.cv2 = Conv((2 + n) * self.c, c2, 1)
        self.m = nn.ModuleList(Bottleneck(self.c, self.c, shortcut) for _ in range(n))

    def forward(self, x):
        y = list(self.cv1(x).chunk(2, 1))
        y.extend(m(y[-1]) for m in self.m)
        return self.cv2(torch.cat(y, 1))


class SPPF(nn.Module):
    def __init__(self, c1, c2, k=5):
        super().__init__()
        c_ = c1 // 2
        self.cv1 = Conv(c1, c_, 1)
        self.cv2 = Conv(c_ * 4, c2, 1)
        self.m = nn.MaxPool2d(k, 1, k // 2)

    def forward(self, x):
        y = [self.cv1(x)]
        y.extend(self.m(y[-1]) for _ in range(3))
        return self.cv2(torch.cat(y, 1))


class DFL(nn.Module):
    def __init__(self, c1=16):
        super().__init__()
        self.conv = nn.Conv2d(c1, 1, 1, bias=False).requires_grad_(False)
        self.conv.weight.data[:] = torch.arange(c1, dtype=torch.float).view(1, c1, 1, 1)
        self.c1 = c1


class Detect(nn.Module):
    def __init__(self, nc, ch):
        super().__init__()
        self.nc, self.reg_max = nc, 16
        c2, c3 = max(16, ch[0] // 4, 64), max(ch[0], min(nc, 100))
        self.cv2 = nn.ModuleList(nn.Sequential(Conv(x, c2, 3), Conv(c2, c2, 3), nn.Conv2d(c2, 64, 1)) for x in ch)
        self.cv3 = nn.ModuleList(nn.Sequential(Conv(x, c3, 3), Conv(c3, c3, 3), nn.Conv2d(c3, nc, 1)) for x in ch)
        self.dfl = DFL(16)

    def forward(self, xs):
        return [torch.cat((self.cv2[i](x), self.cv3[i](x)), 1) for i, x in enumerate(xs)]


class Upsample(nn.Module):
    def forward(self, x):
        return F.interpolate(x, scale_factor=2.0, mode="nearest")


class Concat(nn.Module):
    def forward(self, xs):
        return torch.cat(xs, 1)


class YOLOv8n(nn.Module):
    def __init__(self, nc=1):
        super().__init__()
        self.model = nn.Sequential(
            Conv(3, 16, 3, 2), Conv(16, 32, 3, 2), C2f(32, 32, 1, True), Conv(32, 64, 3, 2), C2f(64, 64, 2, True),
            Conv(64, 128, 3, 2), C2f(128, 128, 2, True), Conv(128, 256, 3, 2), C2f(256, 256, 1, True),
            SPPF(256, 256, 5), Upsample(), Concat(), C2f(384, 128, 1), Upsample(), Concat(), C2f(192, 64, 1),
            Conv(64, 64, 3, 2), Concat(), C2f(192, 128, 1), Conv(128, 128, 3, 2), Concat(), C2f(384, 256, 1),
            Detect(nc, (64, 128, 256)))

    def forward(self, x):
        m = self.model
        y = {}
        x = m[0](x); x = m[1](x); x = m[2](x); x = m[3](x); y[4] = x = m[4](x)
        x = m[5](x); y[6] = x = m[6](x); x = m[7](x); x = m[8](x); y[9] = x = m[9](x)
        x = m[11]([m[10](x), y[6]]); y[12] = x = m[12](x)
        x = m[14]([m[13](x), y[4]]); y[15] = x = m[15](x)
        x = m[17]([m[16](x), y[12]]); y[18] = x = m[18](x)
        x = m[20]([m[19](x), y[9]]); y[21] = x = m[21](x)
        return m[22]([y[15], y[18], y[21]])   # raw per-level [B, 64+nc, H, W]


def build_oracle_yolo(state_dict, nc=1):
    m = YOLOv8n(nc).eval()
    sd = {k: torch.as_tensor(v) for k, v in state_dict.items()}
    missing, unexpected = m.load_state_dict(sd, strict=False)
    missing = [k for k in missing if not k.endswith("num_batches_tracked")]
    if missing or unexpected:
        raise KeyError(f"state_dict mismatch: missing={missing[:5]} unexpected={unexpected[:5]}")
    return m


def raw_heads(levels):
    """[B, 64+nc, A] in level -> (y, x) anchor order (Detect._inference's cat)."""
    return torch.cat([l.flatten(2) for l in levels], 2).numpy()


def decode(raw, shapes, strides=(8, 16, 32)):
    """Per frame: (boxes_xyxy [A,4] in canvas pixels, cls scores [A,nc]) with the
    same float32 op order as the HIP kernel (yolo_candidates_kernel)."""
    B, C, A = raw.shape
    nc = C - 64
    out = []
    ax, ay, st = [], [], []
    for (h, w), s in zip(shapes, strides):
        gy, gx = np.meshgrid(np.arange(h), np.arange(w), indexing="ij")
        ax.append(gx.ravel()); ay.append(gy.ravel()); st.append(np.full(h * w, s))
    ax = np.concatenate(ax).astype(F32) + F32(0.5)
    ay = np.concatenate(ay).astype(F32) + F32(0.5)
    st = np.concatenate(st).astype(F32)
    for b in range(B):
        r = raw[b].T.astype(F32)                                   # [A, 64+nc]
        q = r[:, :64].reshape(A, 4, 16)
        mx = q.max(-1, keepdims=True)
        e = vd_expf(q - mx)
        ssum = np.zeros((A, 4), F32)
        for i in range(16):
            ssum = ssum + e[..., i]
        acc = np.zeros((A, 4), F32)
        for i in range(16):
            acc = acc + (e[..., i] / ssum) * F32(i)
        x1, y1 = ax - acc[:, 0], ay - acc[:, 1]
        x2, y2 = ax + acc[:, 2], ay + acc[:, 3]
        cx = ((x1 + x2) / F32(2)) * st
        cy = ((y1 + y2) / F32(2)) * st
        bw, bh = (x2 - x1) * st, (y2 - y1) * st
        hw, hh = bw / F32(2), bh / F32(2)
        boxes = np.stack([cx - hw, cy - hh, cx + hw, cy + hh], 1).astype(F32)
        cls = (F32(1) / (F32(1) + vd_expf(-r[:, 64:]))).astype(F32)
        out.append((boxes, cls))
    return out


def postprocess(raw, shapes, canvas_hw, img_hw, conf=0.5, iou=0.7, max_det=300, max_wh=7680.0):
    """non_max_suppression + scale_boxes; returns per frame (xyxy float32 [M,4] in
    source pixels, conf [M], class [M], anchor [M])."""
    ch, cw = canvas_hw
    ih, iw = img_hw
    gain = min(ch / ih, cw / iw)
    padx = round((cw - iw * gain) / 2 - 0.1)
    pady = round((ch - ih * gain) / 2 - 0.1)
    inv = F32(1.0) / F32(gain)
    res = []
    for boxes, cls in decode(raw, shapes):
        best = cls.max(1)
        j = cls.argmax(1)
        cand = np.nonzero(best > F32(conf))[0]
        if cand.size == 0:
            res.append((np.zeros((0, 4), F32), np.zeros(0, F32), np.zeros(0, np.int64), np.zeros(0, np.int64)))
            continue
        off = (j[cand].astype(F32) * F32(max_wh)).astype(F32)
        nb = boxes[cand] + off[:, None]
        keep = nms_torchvision(nb, best[cand], iou)[:max_det]
        idx = cand[keep]
        b = boxes[idx].copy()
        b[:, [0, 2]] = (b[:, [0, 2]] - F32(padx)) * inv
        b[:, [1, 3]] = (b[:, [1, 3]] - F32(pady)) * inv
        b[:, [0, 2]] = b[:, [0, 2]].clip(0, iw)
        b[:, [1, 3]] = b[:, [1, 3]].clip(0, ih)
        res.append((b.astype(F32), best[idx], j[idx], idx))
    return res
