"""Synthetic inputs: counter-hash frames and seeded box lists.

``px = splitmix64(key(seed, frame, y, x, c)) & 0xFF`` so the same frame can be
regenerated anywhere without shipping data. Box lists for blur-only timing:
8 boxes/frame, sizes U[24,256] px, ~10 % overlapping, ~5 % partially off-frame.
"""
import numpy as np

_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)
_G = np.uint64(0x9E3779B97F4A7C15)


def splitmix64(x):
    x = np.asarray(x, np.uint64)
    with np.errstate(over="ignore"):
        x = x + _G
        x = (x ^ (x >> np.uint64(30))) * _M1
        x = (x ^ (x >> np.uint64(27))) * _M2
        x = x ^ (x >> np.uint64(31))
    return x


def frame(h, w, index, seed=0):
    """uint8 HxWx3 RGB frame `index`."""
    y = np.arange(h, dtype=np.uint64)[:, None, None]
    x = np.arange(w, dtype=np.uint64)[None, :, None]
    c = np.arange(3, dtype=np.uint64)[None, None, :]
    with np.errstate(over="ignore"):
        key = (((np.uint64(seed) * np.uint64(1000003) + np.uint64(index)) << np.uint64(40))
               ^ (y << np.uint64(20)) ^ (x << np.uint64(2)) ^ c)
    return (splitmix64(key) & np.uint64(0xFF)).astype(np.uint8)


def frames(n, h, w, seed=0, start=0):
    out = np.empty((n, h, w, 3), np.uint8)
    for i in range(n):
        out[i] = frame(h, w, start + i, seed)
    return out


def structured_frames(n, h, w, seed=0, noise=1.5):
    """uint8 [n,h,w,3] frames with the entropy of real video frames: per channel four
    seeded low-frequency plane waves around mid-grey plus N(0, noise) sensor noise
    (~0.45 MB per 1080p frame at JPEG q95 4:2:0, where the counter-hash frames are
    ~2.4 MB). For frame-I/O timing (bench.py jpeg_pipeline_structured)."""
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float32)
    out = np.empty((n, h, w, 3), np.uint8)
    for f in range(n):
        img = np.empty((h, w, 3), np.float32)
        for c in range(3):
            fr = rng.uniform(0.002, 0.02, (4, 2)).astype(np.float32)
            ph = rng.uniform(0, 6.28, 4).astype(np.float32)
            img[..., c] = 128 + sum(40 * np.sin(fr[k, 0] * xx + fr[k, 1] * yy + ph[k]) for k in range(4))
        img += rng.normal(0, noise, (h, w, 1)).astype(np.float32)
        out[f] = np.clip(img, 0, 255).astype(np.uint8)
    return out


def box_lists(n, h, w, per_frame=8, seed=1):
    """int32 [n][per_frame][4] (x1,y1,x2,y2) lists for blur-only runs."""
    rng = np.random.default_rng(seed)
    out = np.zeros((n, per_frame, 4), np.int32)
    for f in range(n):
        for k in range(per_frame):
            bw, bh = rng.integers(24, 257, 2)
            if k > 0 and rng.random() < 0.10:                  # overlap the previous box
                px1, py1 = out[f, k - 1, :2]
                x1 = int(px1 + rng.integers(-bw // 2, bw // 2 + 1))
                y1 = int(py1 + rng.integers(-bh // 2, bh // 2 + 1))
            elif rng.random() < 0.05:                          # partially off-frame
                x1 = int(rng.integers(-bw + 1, w))
                y1 = int(rng.choice([-bh // 2, h - bh // 2]))
            else:
                x1 = int(rng.integers(0, max(1, w - bw)))
                y1 = int(rng.integers(0, max(1, h - bh)))
            out[f, k] = (x1, y1, x1 + bw, y1 + bh)
    return out
