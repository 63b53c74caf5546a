"""Drop-in ``mosaic_rectangle_region_single`` (combine_detect.py:138-161) and the
batched form the MI355X path actually uses (one HIP launch per frame batch,
boxes applied in list order exactly as combine_detect.py:246-249)."""
import threading

import numpy as np

from .context import Context

_ctx = None
_ctx_lock = threading.Lock()


def _default_ctx():
    global _ctx
    with _ctx_lock:
        if _ctx is None:
            _ctx = Context(max_batch=64)
        return _ctx


def mosaic_rectangle_region_single(img, x1, y1, x2, y2, mosaic_level=8):
    """Same signature/result as the reference: returns a new array with the clipped
    box pixelated by an INTER_NEAREST down/up resize of factor ``mosaic_level``."""
    a = np.ascontiguousarray(img, np.uint8)
    box = np.asarray([[[int(x1), int(y1), int(x2), int(y2)]]], np.int32)
    return _default_ctx().mosaic(a[None], box, np.ones(1, np.int32), level=mosaic_level)[0]


def mosaic_frames(frames, boxes, mosaic_level=8, ctx=None):
    """frames: uint8 [n,h,w,3]; boxes: list (per frame) of (x1,y1,x2,y2) int tuples.
    Equivalent to applying mosaic_rectangle_region_single per box in order."""
    frames = np.ascontiguousarray(frames, np.uint8)
    n = frames.shape[0]
    cap = max(1, max((len(b) for b in boxes), default=1))
    xy = np.zeros((n, cap, 4), np.int32)
    cnt = np.zeros(n, np.int32)
    for i, bl in enumerate(boxes):
        cnt[i] = len(bl)
        if len(bl):
            xy[i, :len(bl)] = np.asarray(bl, np.int64).clip(-2**31, 2**31 - 1)
    return (ctx or _default_ctx()).mosaic(frames, xy, cnt, level=mosaic_level)
