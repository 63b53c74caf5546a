"""Generate tests/golden/golden.json from the CPU oracle.

The reference has no tests or vectors and may not be executed
here, so these fixtures pin the oracle against regressions and
give the GPU tests oracle-independent expected values. Inputs are regenerated
from seeds (vdmi.synth counter-hash frames, numpy default_rng), so only seeds,
small inputs and expected outputs (or SHA-256 digests of large outputs) are
stored.

    python tools/make_golden.py
"""
import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "video-desensitization_amd"))

from oracle import anchors, bbox, letterbox, mosaic  # noqa: E402
from vdmi import synth  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden", "golden.json")


def digest(a):
    a = np.ascontiguousarray(a)
    return hashlib.sha256(a.tobytes()).hexdigest()


def post_inputs(seed, bias, A=16800):
    rng = np.random.default_rng(seed)
    loc = (rng.standard_normal((A, 4)) * 1.5).astype(np.float32)
    conf = rng.standard_normal((A, 2)).astype(np.float32)
    conf[:, 1] += np.float32(bias)
    return loc, conf


def mosaic_boxes(seed, h, w, k):
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(k):
        bw, bh = int(rng.integers(1, w // 2)), int(rng.integers(1, h // 2))
        x1, y1 = int(rng.integers(-bw, w)), int(rng.integers(-bh, h))
        out.append([x1, y1, x1 + bw, y1 + bh])
    return out


def main():
    g = {"generator": "tools/make_golden.py (CPU oracle)", "anchors": {}, "letterbox": [], "postprocess": [],
         "mosaic": []}
    a = anchors.get_anchors((640, 640))
    g["anchors"] = {"shape": list(a.shape), "sha256": digest(a), "first": a[:3].tolist(), "last": a[-1].tolist()}
    for (h, w) in [(1080, 1920), (720, 1280), (2160, 3840), (640, 640), (333, 517), (96, 160)]:
        fr = synth.frame(h, w, 0, seed=21)
        x, _ = letterbox.preprocess([fr])
        nhwc = np.ascontiguousarray(x[0].transpose(1, 2, 0))
        g["letterbox"].append({"h": h, "w": w, "frame_seed": 21, "frame_index": 0, "sha256_nhwc_f32": digest(nhwc),
                               "sum": float(nhwc.astype(np.float64).sum())})
    pri = anchors.get_anchors((640, 640))
    for seed, bias, hw in [(1, -4.0, (1080, 1920)), (2, -1.0, (720, 1280)), (3, 0.5, (640, 640))]:
        loc, conf = post_inputs(seed, bias)
        idx, boxes, sc = bbox.postprocess_frame(loc, conf, pri, 0.5, 0.4)
        fb = bbox.correct_and_scale(boxes, *hw)
        g["postprocess"].append({"seed": seed, "bias": bias, "img_hw": list(hw), "kept": idx.tolist(),
                                 "xyxy_f32_sha256": digest(fb),
                                 "xyxy_int_sha256": digest(bbox.truncate_boxes(fb).astype(np.int32)),
                                 "xyxy_int_head": bbox.truncate_boxes(fb)[:8].tolist(),
                                 "score_sha256": digest(sc)})
    for seed, (h, w), k, level in [(4, (120, 160), 12, 8), (5, (1080, 1920), 20, 8), (6, (77, 93), 30, 4)]:
        fr = synth.frame(h, w, 1, seed=seed)
        boxes = mosaic_boxes(seed, h, w, k)
        out = mosaic.mosaic_frame(fr, [tuple(b) for b in boxes], level)
        g["mosaic"].append({"seed": seed, "h": h, "w": w, "frame_index": 1, "level": level, "boxes": boxes,
                            "sha256": digest(out)})
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    with open(OUT, "w") as f:
        json.dump(g, f, indent=1)
    print(OUT, os.path.getsize(OUT), "bytes")


if __name__ == "__main__":
    main()
