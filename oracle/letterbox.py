"""Letterbox + mean subtraction — restates detect_face/utils/utils.py:8-18,27-28 and
Retinaface.preprocess (detect_face/face.py:65-88), with OpenCV 4.9.0.80
``cv2.resize(img, (nw, nh))`` (default INTER_LINEAR, utils/utils.py:15) restated
from upstream imgproc/src/resize.cpp [ext]:

* dsize == ssize                     -> copy;
* integer ratio 2 in both axes       -> INTER_AREA fast path, (a+b+c+d+2)>>2;
* otherwise                          -> fixed-point bilinear, 11-bit coefficients,
  horizontal int pass, vertical pass in the SIMD (VResizeLinearVec_32s8u) form
  ``((mulhi(D0>>4,b0) + mulhi(D1>>4,b1) + 2) >> 2)``.

For the BASELINE configs (640x640, 1280x720, 1920x1080, 3840x2160) every branch
reduces to an exact integer formula, pinned by the
known-answer tests. Other ratios: parity unpinned (OpenCV rounding details).

Also restates the ultralytics LetterBox used by the plate detector [ext]
(auto=True, stride 32, pad value 114, BGR<->RGB flip, /255).
Test infrastructure only.
"""
import numpy as np

MEAN_RGB = np.array((104, 117, 123), np.float32)   # utils/utils.py:28 (applied in RGB order)
COEF_BITS = 11
COEF_SCALE = 1 << COEF_BITS


def letterbox_geometry(ih, iw, size=(640, 640)):
    """utils/utils.py:9-13 in Python doubles: returns (nw, nh, top, left)."""
    w, h = size
    scale = min(w / iw, h / ih)
    nw = int(iw * scale)
    nh = int(ih * scale)
    return nw, nh, (h - nh) // 2, (w - nw) // 2


def _round_half_even_f32_to_short(v):
    # saturate_cast<short>(float) == cvRound == lrintf (round half to even)
    return np.clip(np.rint(v.astype(np.float32)), -32768, 32767).astype(np.int32)


def _linear_taps(dsize, ssize, inv_scale):
    """Per output index: (s0, s1, a0, a1) following resize.cpp's coefficient setup."""
    scale = 1.0 / inv_scale
    d = np.arange(dsize, dtype=np.float64)
    f = ((d + 0.5) * scale - 0.5).astype(np.float32)
    s = np.floor(f).astype(np.int64)
    f = (f - s.astype(np.float32)).astype(np.float32)
    lo = s < 0
    f[lo] = 0.0
    s[lo] = 0
    hi = s >= ssize - 1
    f[hi] = 0.0
    s[hi] = ssize - 1
    a0 = _round_half_even_f32_to_short((np.float32(1.0) - f) * np.float32(COEF_SCALE))
    a1 = _round_half_even_f32_to_short(f * np.float32(COEF_SCALE))
    s1 = np.minimum(s + 1, ssize - 1)
    return s, s1, a0, a1


def cv_resize_linear_u8(img, nw, nh):
    """cv2.resize(img, (nw, nh)) for uint8 HxWxC (default INTER_LINEAR)."""
    ih, iw = img.shape[:2]
    if (nw, nh) == (iw, ih):
        return img.copy()
    inv_sx = nw / iw
    inv_sy = nh / ih
    sx, sy = 1.0 / inv_sx, 1.0 / inv_sy
    isx, isy = int(round(sx)), int(round(sy))
    eps = np.finfo(np.float64).eps
    area_fast = abs(sx - isx) < eps and abs(sy - isy) < eps
    if area_fast and isx == 2 and isy == 2:
        # hal::resize maps INTER_LINEAR at exact 2x to INTER_AREA (resizeAreaFast_)
        a = img[0:2 * nh:2, 0:2 * nw:2].astype(np.int32)
        b = img[0:2 * nh:2, 1:2 * nw:2].astype(np.int32)
        c = img[1:2 * nh:2, 0:2 * nw:2].astype(np.int32)
        d = img[1:2 * nh:2, 1:2 * nw:2].astype(np.int32)
        return ((a + b + c + d + 2) >> 2).astype(np.uint8)
    x0, x1, ax0, ax1 = _linear_taps(nw, iw, inv_sx)
    y0, y1, by0, by1 = _linear_taps(nh, ih, inv_sy)
    src = img.astype(np.int64)
    # horizontal pass (HResizeLinear, int accumulators)
    r0 = src[y0]
    r1 = src[y1]
    d0 = r0[:, x0] * ax0[None, :, None] + r0[:, x1] * ax1[None, :, None]
    d1 = r1[:, x0] * ax0[None, :, None] + r1[:, x1] * ax1[None, :, None]
    # vertical pass, SIMD form (mulhi of int16 lanes)
    t0 = ((d0 >> 4) * by0[:, None, None]) >> 16
    t1 = ((d1 >> 4) * by1[:, None, None]) >> 16
    out = (t0 + t1 + 2) >> 2
    return np.clip(out, 0, 255).astype(np.uint8)


def letterbox_image(img, size=(640, 640)):
    """utils/utils.py:8-18: float64 canvas of 128, resized image pasted centred."""
    ih, iw = img.shape[:2]
    nw, nh, top, left = letterbox_geometry(ih, iw, size)
    w, h = size
    resized = cv_resize_linear_u8(img, nw, nh)
    canvas = np.ones([h, w, 3]) * 128
    canvas[top:top + nh, left:left + nw] = resized
    return canvas


def preprocess(images, size=(640, 640)):
    """face.py:65-88: per image letterbox, subtract (104,117,123) in RGB order,
    HWC->CHW, stack, float32. Returns (NCHW float32, image_shapes float32 [B,2])."""
    tensors, shapes = [], []
    for img in images:
        h, w = img.shape[:2]
        shapes.append([h, w])
        x = letterbox_image(img, size)
        x -= MEAN_RGB        # float64 canvas minus float32 array -> float64 (utils.py:28)
        tensors.append(np.transpose(x, (2, 0, 1)))
    return (np.stack(tensors, 0).astype(np.float32),
            np.asarray(shapes, dtype=np.float32))


# ----------------------------------------------------------------------------
# ultralytics LetterBox (plate detector input) [ext, version unpinned]
# ----------------------------------------------------------------------------
def yolo_letterbox_geometry(ih, iw, imgsz=640, stride=32):
    """LetterBox(new_shape=640, auto=True, stride=32): returns
    (nw, nh, top, left, out_h, out_w)."""
    r = min(imgsz / ih, imgsz / iw)
    nw, nh = int(round(iw * r)), int(round(ih * r))
    dw, dh = imgsz - nw, imgsz - nh
    dw, dh = dw % stride, dh % stride
    dw, dh = dw / 2, dh / 2
    top, bottom = int(round(dh - 0.1)), int(round(dh + 0.1))
    left, right = int(round(dw - 0.1)), int(round(dw + 0.1))
    return nw, nh, top, left, nh + top + bottom, nw + left + right


def yolo_preprocess(images, imgsz=640, stride=32):
    """LetterBox -> copyMakeBorder(114) -> im[..., ::-1] -> /255 -> NCHW float32.
    The reference passes RGB arrays, which ultralytics treats as BGR, so the
    network sees them channel-reversed."""
    outs = []
    for img in images:
        ih, iw = img.shape[:2]
        nw, nh, top, left, oh, ow = yolo_letterbox_geometry(ih, iw, imgsz, stride)
        resized = cv_resize_linear_u8(img, nw, nh) if (nw, nh) != (iw, ih) else img
        canvas = np.full((oh, ow, 3), 114, np.uint8)
        canvas[top:top + nh, left:left + nw] = resized
        x = canvas[..., ::-1].transpose(2, 0, 1).astype(np.float32) / np.float32(255.0)
        outs.append(x)
    return np.stack(outs, 0)
