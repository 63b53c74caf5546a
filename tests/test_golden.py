"""Golden fixtures (tests/golden/golden.json, made by tools/make_golden.py):
the CPU oracle must reproduce them (CPU), and so must the HIP path (GPU),
bit for bit, without consulting the oracle at run time."""
import json
import os
import sys

import numpy as np
import pytest

from conftest import GOLDEN, ROOT

sys.path.insert(0, os.path.join(ROOT, "tools"))
import make_golden as mg  # noqa: E402

G = json.load(open(os.path.join(GOLDEN, "golden.json")))


def test_oracle_anchors_golden():
    from oracle import anchors
    a = anchors.get_anchors((640, 640))
    assert mg.digest(a) == G["anchors"]["sha256"]


@pytest.mark.parametrize("case", G["letterbox"], ids=lambda c: f"{c['w']}x{c['h']}")
def test_oracle_letterbox_golden(case):
    from oracle import letterbox
    from vdmi import synth
    fr = synth.frame(case["h"], case["w"], case["frame_index"], seed=case["frame_seed"])
    x, _ = letterbox.preprocess([fr])
    assert mg.digest(np.ascontiguousarray(x[0].transpose(1, 2, 0))) == case["sha256_nhwc_f32"]


@pytest.mark.parametrize("case", G["postprocess"], ids=lambda c: f"seed{c['seed']}")
def test_oracle_postprocess_golden(case):
    from oracle import anchors, bbox
    loc, conf = mg.post_inputs(case["seed"], case["bias"])
    idx, boxes, sc = bbox.postprocess_frame(loc, conf, anchors.get_anchors((640, 640)), 0.5, 0.4)
    fb = bbox.correct_and_scale(boxes, *case["img_hw"])
    assert idx.tolist() == case["kept"]
    assert mg.digest(fb) == case["xyxy_f32_sha256"]
    ib = bbox.truncate_boxes(fb)
    assert mg.digest(ib.astype(np.int32)) == case["xyxy_int_sha256"] and ib[:8].tolist() == case["xyxy_int_head"]


@pytest.mark.parametrize("case", G["mosaic"], ids=lambda c: f"seed{c['seed']}")
def test_oracle_mosaic_golden(case):
    from oracle import mosaic
    from vdmi import synth
    fr = synth.frame(case["h"], case["w"], case["frame_index"], seed=case["seed"])
    out = mosaic.mosaic_frame(fr, [tuple(b) for b in case["boxes"]], case["level"])
    assert mg.digest(out) == case["sha256"]


# ------------------------------------------------------------------ GPU vs fixtures
@pytest.mark.gpu
@pytest.mark.parametrize("case", G["letterbox"], ids=lambda c: f"{c['w']}x{c['h']}")
def test_gpu_letterbox_golden(gpu, face_ctx_factory, case):
    from vdmi import synth
    fr = synth.frame(case["h"], case["w"], case["frame_index"], seed=case["frame_seed"])
    got = face_ctx_factory("fp32", 8).letterbox(fr[None], cpad=3)[0]
    assert mg.digest(got) == case["sha256_nhwc_f32"]


@pytest.mark.gpu
@pytest.mark.parametrize("case", G["postprocess"], ids=lambda c: f"seed{c['seed']}")
def test_gpu_postprocess_golden(gpu, face_ctx_factory, case):
    loc, conf = mg.post_inputs(case["seed"], case["bias"])
    got = face_ctx_factory("fp32", 8).postprocess(loc[None], conf[None], case["img_hw"], cap=16800)
    xi, xf, sc, lab = got.frame(0)
    assert lab.tolist() == case["kept"]
    assert mg.digest(xf) == case["xyxy_f32_sha256"]
    assert mg.digest(xi.astype(np.int32)) == case["xyxy_int_sha256"] and xi[:8].tolist() == case["xyxy_int_head"]
    assert mg.digest(sc) == case["score_sha256"]


@pytest.mark.gpu
@pytest.mark.parametrize("case", G["mosaic"], ids=lambda c: f"seed{c['seed']}")
def test_gpu_mosaic_golden(gpu, face_ctx_factory, case):
    from vdmi import mosaic_frames, synth
    fr = synth.frame(case["h"], case["w"], case["frame_index"], seed=case["seed"])
    out = mosaic_frames(fr[None], [[tuple(b) for b in case["boxes"]]], case["level"], ctx=face_ctx_factory("bf16", 8))
    assert mg.digest(out[0]) == case["sha256"]
