"""Print where the GPU mosaic differs from the oracle on a golden mosaic case."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "video-desensitization_amd"))
import numpy as np  # noqa: E402
from oracle import mosaic as om  # noqa: E402
import vdmi  # noqa: E402
from vdmi import mosaic_frames, synth  # noqa: E402

G = json.load(open(os.path.join(ROOT, "tests", "golden", "golden.json")))
ctx = vdmi.Context(device=0, precision="bf16", max_batch=8)
for case in G["mosaic"]:
    fr = synth.frame(case["h"], case["w"], case["frame_index"], seed=case["seed"])
    boxes = [tuple(b) for b in case["boxes"]]
    got = mosaic_frames(fr[None], [boxes], case["level"], ctx=ctx)[0]
    exp = om.mosaic_frame(fr, boxes, case["level"])
    bad = np.argwhere((got != exp).any(-1))
    print("seed", case["seed"], "mismatched pixels", len(bad))
    if len(bad):
        ys, xs = bad[:, 0], bad[:, 1]
        print(" rows", np.unique(ys)[:40], "\n cols", np.unique(xs)[:60])
        for y, x in bad[:10]:
            print(" ", y, x, got[y, x], exp[y, x], fr[y, x])
