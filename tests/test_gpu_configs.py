"""BASELINE.json configs at their own sizes (the bench runs config 3; these are
the parity cases for the others and full-batch properties of config 3).

* C2 (RetinaFace + blur, B=32, 1280x720, bf16): heads and boxes against the
  oracle on a sample of frames; the whole B=32 vd_process mosaic exact given
  its complete box lists.
* C3 (B=64, 1920x1080, faces + plates): every frame's mosaic exact given its
  complete box lists, in fp32 (the headline) and bf16; the measured fraction of
  frames whose bf16 / fp16 keep lists equal the fp32 path's (the bench's
  `parity` block) asserted against a floor.
* C5 single-GPU slice (3840x2160, fp16): vd_process with mosaic on 4K frames,
  pixels exact given boxes (11 520-byte rows through the band/vector logic of
  mosaic_out_kernel); boxes against the oracle.
"""
import numpy as np
import pytest
import torch

from oracle import anchors as oanchors
from oracle import bbox as obbox
from oracle import letterbox as olb
from oracle import mosaic as omosaic
from oracle.retinaface import build_oracle_model

from conftest import face_weights

pytestmark = pytest.mark.gpu


def _frames(n, h, w, seed=0):
    from vdmi import synth
    return synth.frames(n, h, w, seed=seed)


def _frames720(n, seed):
    """1280x720 frames that are 2x nearest upsamples of 640x360 synthetic frames: the
    ratio-2 area letterbox then recovers the 640x360 structure exactly, so the
    calibrated random weights fire (raw 720p noise averages out to no faces)."""
    return np.repeat(np.repeat(_frames(n, 360, 640, seed=seed), 2, axis=1), 2, axis=2)


def _rel(a, b):
    return np.abs(a - b).max() / (np.abs(b).max() + 1e-12)


def _oracle_heads(frames):
    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
    m = build_oracle_model(face_weights("default"))
    x, _ = olb.preprocess(list(frames))
    with torch.no_grad():
        loc, cls, _ = m.forward_raw(torch.from_numpy(x))
    return loc.numpy(), cls.numpy()


def _complete(ctx, net, n):
    b = ctx.read_boxes(net, n)
    return [(b.label[i, :b.count[i]].copy(), b.xyxy[i, :b.count[i]].copy()) for i in range(n)]


def _mosaic_exact(frames, out, lists_faces, lists_plates=None):
    for i in range(frames.shape[0]):
        boxes = [tuple(int(v) for v in r) for r in lists_faces[i][1]]
        if lists_plates is not None:
            boxes += [tuple(int(v) for v in r) for r in lists_plates[i][1]]
        exp = omosaic.mosaic_frame(frames[i], boxes, 8)
        assert np.array_equal(out[i], exp), f"frame {i}: mosaic differs from the oracle given its boxes"


def _iou_match(e, g, thr=0.9):
    matched = 0
    for r in e:
        if len(g) == 0:
            break
        x1 = np.maximum(r[0], g[:, 0]); y1 = np.maximum(r[1], g[:, 1])
        x2 = np.minimum(r[2], g[:, 2]); y2 = np.minimum(r[3], g[:, 3])
        inter = np.clip(x2 - x1, 0, None) * np.clip(y2 - y1, 0, None)
        iou = inter / ((r[2] - r[0]) * (r[3] - r[1]) + (g[:, 2] - g[:, 0]) * (g[:, 3] - g[:, 1]) - inter)
        matched += iou.max() >= thr
    return matched


# ------------------------------------------------------------------ C2
# bf16 C2 box agreement with the f32 oracle over the 32 frames of seed 31: (batch share,
# worst frame share) floors; measured 893/928 = 0.962 and 0.792 (r04 GPU run)
C2_BOX_FLOOR = (0.93, 0.75)


def test_c2_bf16_720p_heads_and_boxes(gpu, face_ctx_factory):
    """bf16 at 1280x720 (ratio-2 area letterbox), the whole C2 batch of 32 frames: heads
    within the bf16 bound, and the share of oracle boxes matched at IoU >= 0.9 above
    its measured floor (C2_BOX_FLOOR), per batch and per frame."""
    ctx = face_ctx_factory("bf16", 32)
    fr = _frames720(32, seed=31)
    loc, conf, _ = ctx.forward_heads(fr)
    eloc, econf = _oracle_heads(fr)
    assert _rel(loc, eloc) < 2e-2 and _rel(conf, econf) < 2e-2      # observed <= 0.0116 (~1.5x)
    got = ctx.detect(fr)
    pri = oanchors.get_anchors((640, 640))
    matched = total = 0
    worst = 1.0
    for b in range(32):
        _, boxes, _ = obbox.postprocess_frame(eloc[b], econf[b], pri, 0.5, 0.4)
        e = obbox.correct_and_scale(boxes, 720, 1280)
        mb = _iou_match(e, got.frame(b)[1])
        total += len(e)
        matched += mb
        if len(e):
            worst = min(worst, mb / len(e))
    print(f"C2 bf16 boxes matched at IoU >= 0.9: {matched}/{total}, worst frame {worst:.3f}")
    assert total > 0 and matched / total >= C2_BOX_FLOOR[0], (matched, total)
    assert worst >= C2_BOX_FLOOR[1], worst


def test_c2_bf16_720p_b32_process_mosaic_exact(gpu):
    import vdmi
    from vdmi import _lib
    ctx = vdmi.Context(precision="bf16", max_batch=32)
    try:
        ctx.load_weights(0, face_weights("default"))
        fr = _frames720(32, seed=32)
        out, faces, _ = ctx.process(fr)
        lists = _complete(ctx, _lib.VD_NET_RETINAFACE, 32)
        assert sum(len(l[0]) for l in lists) > 0
        _mosaic_exact(fr, out, lists)
    finally:
        ctx.close()


# ------------------------------------------------------------------ C3
@pytest.fixture(scope="module")
def c3_runs(gpu):
    """B=64 1080p faces + plates (MOSAIC_PLATES: every pixel path exercised), one
    run per precision on the same device-resident frames."""
    import vdmi
    from vdmi import _lib, weights
    fr = _frames(64, 1080, 1920, seed=0)
    dev = torch.device("cuda:0")
    dfr = torch.from_numpy(fr).to(dev)
    flags = _lib.VD_PROC_FACES | _lib.VD_PROC_PLATES | _lib.VD_PROC_MOSAIC | _lib.VD_PROC_MOSAIC_PLATES
    runs = {}
    for prec in ("fp32", "bf16", "fp16"):
        ctx = vdmi.Context(precision=prec, max_batch=64)
        try:
            ctx.load_weights(0, face_weights("default"))
            ctx.load_weights(1, weights.yolov8n_state_dict(0))
            out, _, _ = ctx.process(dfr, faces=vdmi.DeviceBoxes(64, 256, dev),
                                    plates=vdmi.DeviceBoxes(64, 256, dev), flags=flags)
            torch.cuda.synchronize()
            runs[prec] = (out.cpu().numpy(), _complete(ctx, _lib.VD_NET_RETINAFACE, 64),
                          _complete(ctx, _lib.VD_NET_YOLOV8N, 64))
        finally:
            ctx.close()
    return fr, runs


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
def test_c3_b64_mosaic_exact_given_boxes(c3_runs, prec):
    fr, runs = c3_runs
    out, faces, plates = runs[prec]
    assert sum(len(l[0]) for l in faces) > 0 and sum(len(l[0]) for l in plates) > 0
    _mosaic_exact(fr, out, faces, plates)


def _agree(a, b):
    return sum(np.array_equal(x[0], y[0]) and np.array_equal(x[1], y[1]) for x, y in zip(a, b)) / len(a)


# Floors, measured on the B=64 bench frames (r03 GPU run, printed by the test) minus a
# margin for box-to-box variation: the fraction of fp32 face boxes that a 16-bit box
# matches at IoU >= 0.9. (Identical keep lists are rare in 16 bits -- ~30 faces per
# frame with seeded weights, so one moved near-threshold box flips a frame -- and
# that fraction is printed, not asserted: box-index parity is an fp32-plan claim.)
# r03: bf16 1895/1964 = 0.965, fp16 1944/1964 = 0.990 (0/64 frames identical in either)
IOU09_FLOOR = {"bf16": 0.94, "fp16": 0.975}


@pytest.mark.parametrize("prec", ["bf16", "fp16"])
def test_c3_b64_keep_list_agreement_with_fp32(c3_runs, prec):
    """Measured, not assumed: the fraction of fp32 boxes over B=64 frames that the
    16-bit path reproduces at IoU >= 0.9, against a floor; plus the fraction of frames
    whose complete keep lists and int boxes are identical (reported)."""
    _, runs = c3_runs
    f32, other = runs["fp32"][1], runs[prec][1]
    frac = _agree(other, f32)
    total = matched = 0
    for x, y in zip(f32, other):
        total += len(x[1])
        matched += _iou_match(x[1].astype(np.float64), y[1].astype(np.float64), 0.9)
    m09 = matched / max(total, 1)
    print(f"{prec} vs fp32: {frac:.3f} of 64 frames identical; {matched}/{total} = {m09:.4f} of fp32 boxes "
          f"matched at IoU >= 0.9")
    assert total > 0 and m09 >= IOU09_FLOOR[prec], (matched, total)


# ------------------------------------------------------------------ C5 (one GPU)
def test_c5_fp16_4k_process_mosaic_and_boxes(gpu):
    """fp16 4K: the 4K frames are 2x nearest upsamples of 1080p synthetic frames (so
    the ratio-6 letterbox sees structure and the calibrated weights fire). Pixels
    exact given the complete box lists; boxes match the oracle's at IoU >= 0.9."""
    import vdmi
    from vdmi import _lib
    fr = np.repeat(np.repeat(_frames(4, 1080, 1920, seed=17), 2, axis=1), 2, axis=2)
    ctx = vdmi.Context(precision="fp16", max_batch=4)
    try:
        ctx.load_weights(0, face_weights("default"))
        out, faces, _ = ctx.process(fr)
        lists = _complete(ctx, _lib.VD_NET_RETINAFACE, 4)
    finally:
        ctx.close()
    assert sum(len(l[0]) for l in lists) > 0
    _mosaic_exact(fr, out, lists)
    eloc, econf = _oracle_heads(fr[:2])
    pri = oanchors.get_anchors((640, 640))
    matched = total = 0
    for b in range(2):
        _, boxes, _ = obbox.postprocess_frame(eloc[b], econf[b], pri, 0.5, 0.4)
        e = obbox.correct_and_scale(boxes, 2160, 3840)
        total += len(e)
        matched += _iou_match(e, faces.frame(b)[1])
    assert total > 0 and matched / total >= 0.95, (matched, total)
