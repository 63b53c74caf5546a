"""SSD prior boxes — restates detect_face/utils/anchors.py:7-41 with cfg_re50
(detect_face/utils/config.py:18-29). Test infrastructure only (see oracle/__init__.py)."""
from math import ceil

import numpy as np

MIN_SIZES = ((16, 32), (64, 128), (256, 512))   # config.py:20
STEPS = (8, 16, 32)                              # config.py:21
VARIANCE = (0.1, 0.2)                            # config.py:22


def get_anchors(image_size=(640, 640)):
    """anchors.py:20 feature maps = ceil(size/step); anchors.py:29-36 order is
    level -> i (row) -> j (col) -> min_size; values computed in Python doubles
    and rounded to float32 by ``torch.Tensor(list)`` (anchors.py:38); clip=False."""
    ih, iw = image_size
    out = []
    for k, step in enumerate(STEPS):
        fh, fw = ceil(ih / step), ceil(iw / step)
        for i in range(fh):
            for j in range(fw):
                for ms in MIN_SIZES[k]:
                    s_kx = ms / iw
                    s_ky = ms / ih
                    cx = (j + 0.5) * step / iw
                    cy = (i + 0.5) * step / ih
                    out.append((cx, cy, s_kx, s_ky))
    return np.asarray(out, dtype=np.float64).astype(np.float32)


def level_offsets(image_size=(640, 640)):
    """First anchor index of each FPN level (heads concat order, retinaface.py:140-142)."""
    ih, iw = image_size
    offs, n = [], 0
    for step in STEPS:
        offs.append(n)
        n += ceil(ih / step) * ceil(iw / step) * 2
    return offs, n
