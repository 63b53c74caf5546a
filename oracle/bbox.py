"""Decode, score, NMS, box correction and int() truncation — restated in numpy
float32 with the reference's operation order. Test infrastructure only.

Sources: detect_face/utils/utils_bbox.py:12-43 (correct boxes), :49-59 (decode),
:64-79 (decode_landm), :103-130 (non_max_suppression -> torchvision
batched_nms [ext]); detect_face/retinaface.py:147 (eval softmax);
detect_face/face.py:93-115 (postprocess), :136-148 (scale by [w,h,w,h]);
combine_detect.py:243 (int()).
"""
import numpy as np

from .vdexp import vd_expf

F32 = np.float32


def softmax2(conf_logits):
    """retinaface.py:147 ``F.softmax(classifications, dim=-1)`` over 2 classes:
    m = max, e_k = exp(x_k - m), p_k = e_k / (e_0 + e_1)  (float32)."""
    c = np.asarray(conf_logits, F32)
    m = np.maximum(c[..., 0], c[..., 1])
    e0 = vd_expf(c[..., 0] - m)
    e1 = vd_expf(c[..., 1] - m)
    s = e0 + e1
    return np.stack([e0 / s, e1 / s], -1).astype(F32)


def softmax2_torch(conf_logits, form="divide"):
    """retinaface.py:147 with torch's own exp instead of the shared ``vd_expf``
    restatement -- measurement only (tools/exp_substitution.py). form "divide": the
    softmax2 formula (max, exp, e_k / sum: the form of torch's CUDA softmax for short
    rows, which is where the reference runs it -- its CPU path raises at
    utils_bbox.py's unconditional .cuda()) with ``torch.exp`` (CPU, SLEEF); form
    "torch": ``torch.softmax`` on the CPU as-is (it multiplies by 1 / sum)."""
    import torch
    c = torch.from_numpy(np.ascontiguousarray(conf_logits, F32))
    if form == "torch":
        return torch.softmax(c, dim=-1).numpy()
    m = torch.maximum(c[..., 0], c[..., 1])
    e0, e1 = torch.exp(c[..., 0] - m), torch.exp(c[..., 1] - m)
    s = e0 + e1
    return torch.stack([e0 / s, e1 / s], -1).numpy()


def decode_torch(loc, priors, variances=(0.1, 0.2)):
    """utils_bbox.py:49-59 as the reference writes it, in torch-CPU ops (``torch.exp``):
    cat(p_xy + loc_xy * v0 * p_wh, p_wh * exp(loc_wh * v1)); xy1 -= wh / 2; xy2 += xy1."""
    import torch
    lo = torch.from_numpy(np.ascontiguousarray(loc, F32))
    p = torch.from_numpy(np.ascontiguousarray(priors, F32))
    b = torch.cat((p[:, :2] + lo[:, :2] * variances[0] * p[:, 2:], p[:, 2:] * torch.exp(lo[:, 2:] * variances[1])), 1)
    b[:, :2] -= b[:, 2:] / 2
    b[:, 2:] += b[:, :2]
    return b.numpy()


def decode(loc, priors, variances=(0.1, 0.2)):
    """utils_bbox.py:49-59. Python-float variances act as float32 scalars.
    cx = p_cx + (l*0.1)*p_w ; w = p_w*exp(l*0.2) ; x1 = cx - w/2 ; x2 = w + x1."""
    loc = np.asarray(loc, F32)
    p = np.asarray(priors, F32)
    v0, v1 = F32(variances[0]), F32(variances[1])
    cxcy = p[..., :2] + (loc[..., :2] * v0) * p[..., 2:]
    wh = p[..., 2:] * vd_expf(loc[..., 2:] * v1)
    xy1 = cxcy - wh / F32(2)
    xy2 = wh + xy1
    return np.concatenate([xy1, xy2], -1).astype(F32)


def decode_landm(landm, priors, variances=(0.1, 0.2)):
    """utils_bbox.py:64-79 (computed and discarded by the driver, face.py:146)."""
    landm = np.asarray(landm, F32)
    p = np.asarray(priors, F32)
    v0 = F32(variances[0])
    parts = [p[..., :2] + (landm[..., 2 * i:2 * i + 2] * v0) * p[..., 2:] for i in range(5)]
    return np.concatenate(parts, -1).astype(F32)


def nms_torchvision(boxes, scores, iou_threshold):
    """torchvision.ops.nms CPU kernel semantics [ext, torchvision 0.22.1]:
    stable descending sort; area = (x2-x1)*(y2-y1); inter = max(0,w)*max(0,h);
    ovr = inter / ((area_i + area_j) - inter) in float32; suppress j when
    ``(double)ovr > iou_threshold`` (threshold kept as a double). Returns the
    kept indices in descending-score order."""
    boxes = np.asarray(boxes, F32)
    scores = np.asarray(scores, F32)
    n = boxes.shape[0]
    if n == 0:
        return np.zeros((0,), np.int64)
    x1, y1, x2, y2 = boxes[:, 0], boxes[:, 1], boxes[:, 2], boxes[:, 3]
    areas = (x2 - x1) * (y2 - y1)
    order = np.argsort(-scores, kind="stable")
    suppressed = np.zeros(n, bool)
    keep = []
    thr = float(iou_threshold)
    zero = F32(0)
    for pos in range(n):
        i = order[pos]
        if suppressed[i]:
            continue
        keep.append(i)
        rest = order[pos + 1:]
        rest = rest[~suppressed[rest]]
        if rest.size == 0:
            continue
        xx1 = np.maximum(x1[i], x1[rest])
        yy1 = np.maximum(y1[i], y1[rest])
        xx2 = np.minimum(x2[i], x2[rest])
        yy2 = np.minimum(y2[i], y2[rest])
        w = np.maximum(zero, xx2 - xx1)
        h = np.maximum(zero, yy2 - yy1)
        inter = w * h
        with np.errstate(invalid="ignore", divide="ignore"):
            ovr = inter / ((areas[i] + areas[rest]) - inter)
        suppressed[rest[ovr.astype(np.float64) > thr]] = True
    return np.asarray(keep, np.int64)


def scores_boxes(loc, conf_logits, anchors, torch_exp=None):
    """(face score [A], decoded boxes [A,4]) of one frame. torch_exp None: vd_expf
    (the restatement the device twins); "divide" / "torch": torch's exp (decode_torch,
    softmax2_torch(form)) -- measurement only."""
    if torch_exp:
        return softmax2_torch(conf_logits, torch_exp)[:, 1], decode_torch(loc, anchors)
    return softmax2(conf_logits)[:, 1], decode(loc, anchors)


def postprocess_frame(loc, conf_logits, anchors, conf_thres=0.5, nms_iou=0.4, torch_exp=None):
    """One image of face.py:93-115 up to (not including) box correction.
    Returns (anchor_idx [M] int64 in output order, boxes [M,4] float32 normalised,
    scores [M] float32). torch_exp: see scores_boxes (measurement only)."""
    score, boxes = scores_boxes(loc, conf_logits, anchors, torch_exp)
    cand = np.nonzero(score >= F32(conf_thres))[0]      # utils_bbox.py:115-116 (>=, inclusive)
    if cand.size == 0:
        return np.zeros((0,), np.int64), np.zeros((0, 4), F32), np.zeros((0,), F32)
    keep = nms_torchvision(boxes[cand], score[cand], nms_iou)   # utils_bbox.py:121-127
    idx = cand[keep]
    return idx, boxes[idx], score[idx]


def correct_factors(img_h, img_w, input_shape=(640, 640)):
    """utils_bbox.py:118-132 in float32 tensors: returns (offset_xy, scale_xy)."""
    inp = np.asarray(input_shape, F32)                 # [H, W]
    ish = np.asarray([img_h, img_w], F32)
    new_shape = ish * np.min(inp / ish)
    offset = (inp - new_shape) / F32(2.0) / inp
    scale = inp / new_shape
    return (np.asarray([offset[1], offset[0]], F32), np.asarray([scale[1], scale[0]], F32))


def correct_and_scale(boxes, img_h, img_w, input_shape=(640, 640)):
    """utils_bbox.py:137 ``(box - offset) * scale`` then face.py:144-145
    ``*= [w, h, w, h]`` (float32 numpy). Returns float32 source-pixel boxes."""
    boxes = np.asarray(boxes, F32)
    off, sc = correct_factors(img_h, img_w, input_shape)
    off4 = np.concatenate([off, off])
    sc4 = np.concatenate([sc, sc])
    b = (boxes - off4) * sc4
    whwh = np.asarray([img_w, img_h, img_w, img_h], F32)
    return (b * whwh).astype(F32)


def truncate_boxes(boxes_f32):
    """combine_detect.py:243 ``int(x)`` on Python floats: truncation toward zero."""
    return np.trunc(np.asarray(boxes_f32, np.float64)).astype(np.int64)
