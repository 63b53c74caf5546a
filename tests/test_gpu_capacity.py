"""Crowded frames: more kept faces than the caller's box capacity.

The reference blurs EVERY kept box (combine_detect.py:241-249, no cap). The
library keeps each frame's complete keep list internally; the mosaic of
vd_process reads that list, never the caller's cap-limited copy, and the
caller's count is the complete count (vd_read_boxes returns the rest).

Weights: the reference keys with zeroed box/class head weights, so every head
output is its bias exactly in every precision (loc = 0 -> boxes are the priors;
class-1 logit +5 on level 0 -> all 12 800 level-0 anchors are candidates and
NMS keeps thousands per frame). The expected boxes come from the oracle's
post-processing of those exact heads, the expected pixels from the oracle's
sequential mosaic over the complete list.
"""
import numpy as np
import pytest

from oracle import anchors as oanchors
from oracle import bbox as obbox
from oracle import mosaic as omosaic

pytestmark = pytest.mark.gpu
F32 = np.float32


def _crowd_weights():
    from vdmi import weights
    sd = weights.retinaface_state_dict(0)
    for lvl in range(3):
        sd[f"BboxHead.{lvl}.conv1x1.weight"][:] = 0
        sd[f"BboxHead.{lvl}.conv1x1.bias"][:] = 0
        sd[f"ClassHead.{lvl}.conv1x1.weight"][:] = 0
        b = np.zeros(4, F32)
        b[1] = b[3] = 5.0 if lvl == 0 else -5.0
        sd[f"ClassHead.{lvl}.conv1x1.bias"] = b
    return sd


def _expected(n, h, w):
    pri = oanchors.get_anchors((640, 640))
    A = pri.shape[0]
    loc = np.zeros((A, 4), F32)
    conf = np.zeros((A, 2), F32)
    conf[:12800, 1] = 5.0
    conf[12800:, 1] = -5.0
    idx, boxes, _ = obbox.postprocess_frame(loc, conf, pri, 0.5, 0.4)
    ib = obbox.truncate_boxes(obbox.correct_and_scale(boxes, h, w))
    return idx, ib


@pytest.fixture(scope="module")
def crowd_ctx(gpu):
    import vdmi
    ctx = vdmi.Context(precision="bf16", max_batch=4, max_boxes=256)
    ctx.load_weights(0, _crowd_weights())
    yield ctx
    ctx.close()


@pytest.mark.parametrize("where", ["device", "host"])
def test_mosaic_covers_every_kept_box_past_cap(crowd_ctx, where):
    import torch
    import vdmi
    from vdmi import _lib, synth
    n, h, w = 2, 320, 320
    frames = synth.frames(n, h, w, seed=7)
    e_idx, e_ib = _expected(n, h, w)
    assert len(e_idx) > 256
    cap = 256
    if where == "device":
        dev = torch.device("cuda:0")
        fr = torch.from_numpy(frames).to(dev)
        faces = vdmi.DeviceBoxes(n, cap, dev)
        out, faces, _ = crowd_ctx.process(fr, faces=faces)
        torch.cuda.synchronize()
        out = out.cpu().numpy()
        count = faces.count.cpu().numpy()
        lab = faces.label.cpu().numpy()
    else:
        faces = _lib.HostBoxes(n, cap)
        out, faces, _ = crowd_ctx.process(frames, faces=faces)   # explicit cap: no auto re-read
        count, lab = faces.count, faces.label
    for b in range(n):
        assert int(count[b]) == len(e_idx)                      # complete count, not min(count, cap)
        np.testing.assert_array_equal(lab[b, :cap], e_idx[:cap])
        full = crowd_ctx.read_boxes(_lib.VD_NET_RETINAFACE, n)
        np.testing.assert_array_equal(full.frame(b)[3], e_idx)
        np.testing.assert_array_equal(full.frame(b)[0], e_ib)
        exp = omosaic.mosaic_frame(frames[b], [tuple(int(v) for v in r) for r in e_ib], 8)
        assert np.array_equal(out[b], exp), f"frame {b}: mosaic differs from the complete-list oracle"


def test_auto_boxes_are_complete(crowd_ctx):
    """Library-allocated host lists (boxes=None) come back complete (re-read past max_boxes)."""
    from vdmi import synth
    frames = synth.frames(1, 320, 320, seed=3)
    e_idx, e_ib = _expected(1, 320, 320)
    faces = crowd_ctx.detect(frames)
    assert faces.cap >= len(e_idx) and int(faces.count[0]) == len(e_idx)
    np.testing.assert_array_equal(faces.frame(0)[3], e_idx)
    np.testing.assert_array_equal(faces.frame(0)[0], e_ib)


def test_host_mosaic_refuses_truncated_list(crowd_ctx):
    """vd_mosaic on a host list whose count exceeds its cap is an error, never a silent skip."""
    import vdmi
    from vdmi import synth
    frames = synth.frames(1, 64, 64, seed=1)
    xy = np.zeros((1, 2, 4), np.int32)
    with pytest.raises(vdmi.VdCapacityError):
        crowd_ctx.mosaic(frames, xy, np.array([3], np.int32))
