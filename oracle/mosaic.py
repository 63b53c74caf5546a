"""Pixelation mosaic — restates combine_detect.py:138-161 (``mosaic_rectangle_region_single``)
and its sequential application per box at combine_detect.py:235-251, with
OpenCV ``resizeNN`` [ext, 4.9.0.80]: for dst size D from src size S,
``src = min(floor(d * (1.0 / ((double)D / S))), S - 1)`` (double arithmetic).
Integer/gather only, so parity is exact. Test infrastructure only.
"""
import numpy as np


def nn_map(dst, src):
    """resize.cpp resizeNN offsets: ifx = 1./fx with fx = (double)dst/src."""
    ifx = 1.0 / (float(dst) / float(src))
    d = np.arange(dst, dtype=np.float64)
    return np.minimum(np.floor(d * ifx).astype(np.int64), src - 1)


def mosaic_axis_map(b, level=8):
    """Composite down(up(x)) map over one axis of a clipped box of size b:
    out[x] = area[down[up[x]]] (combine_detect.py:152-158)."""
    s = max(1, b // level)
    down = nn_map(s, b)     # small[x'] = area[down[x']]
    up = nn_map(b, s)       # out[x]   = small[up[x]]
    return down[up]


def mosaic_rectangle_region_single(img, x1, y1, x2, y2, mosaic_level=8):
    """combine_detect.py:138-161 (new array returned, input untouched)."""
    img = img.copy()
    h, w = img.shape[:2]
    x1 = max(0, x1)
    y1 = max(0, y1)
    x2 = min(w, x2)
    y2 = min(h, y2)
    if x2 <= x1 or y2 <= y1:
        return img
    mx = mosaic_axis_map(x2 - x1, mosaic_level)
    my = mosaic_axis_map(y2 - y1, mosaic_level)
    area = img[y1:y2, x1:x2]
    img[y1:y2, x1:x2] = area[my][:, mx]
    return img


def mosaic_frame(img, boxes, mosaic_level=8):
    """combine_detect.py:246-249: boxes applied in list order, each reading the
    previous box's output. ``boxes`` are Python-int (x1,y1,x2,y2) tuples.
    One copy of the frame, then each box rewrites its region from the current
    state -- the same values as the reference's fresh array per box
    (mosaic_rectangle_region_single), without a full-frame copy per box
    (checked against that composition in tests/test_oracle_kat.py)."""
    out = img.copy()
    h, w = out.shape[:2]
    for (x1, y1, x2, y2) in boxes:
        x1, y1, x2, y2 = max(0, int(x1)), max(0, int(y1)), min(w, int(x2)), min(h, int(y2))
        if x2 <= x1 or y2 <= y1:
            continue
        mx = mosaic_axis_map(x2 - x1, mosaic_level)
        my = mosaic_axis_map(y2 - y1, mosaic_level)
        out[y1:y2, x1:x2] = out[y1:y2, x1:x2][my][:, mx]   # fancy indexing reads a copy first
    return out
