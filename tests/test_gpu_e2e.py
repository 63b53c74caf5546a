"""End-to-end parity: letterbox -> RetinaFace forward -> decode/NMS -> correction ->
int() -> mosaic, GPU (C-ABI) vs the CPU oracle on identical synthetic frames.

* fp32 mode: heads and every frame's boxes against the oracle at every config size
  live in tests/test_gpu_parity_fp32.py (run first); here: mosaic pixels bit-exact
  given the boxes, the drop-in surface, and fused-vs-unfused A/B checks.
* bf16 mode: heads within 2e-2 (R50) / 4.5e-2 (MobileNet) relative, ~1.5x the observed
  error; >= 90 % of oracle boxes matched by a
  GPU box at IoU >= 0.9 (bf16 rounding moves near-threshold decisions, so box
  parity is claimed for fp32 mode only).
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
F32 = np.float32

_ORACLE = {}


def _oracle_heads(frames, wkind="default"):
    key = (wkind, frames.shape, int(frames[:, ::97, ::89].sum()))
    if key not in _ORACLE:
        torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
        m = build_oracle_model(face_weights(wkind))
        x, _ = olb.preprocess(list(frames))
        with torch.no_grad():
            loc, cls, ldm = m.forward_raw(torch.from_numpy(x))
        _ORACLE[key] = (loc.numpy(), cls.numpy(), ldm.numpy())
    return _ORACLE[key]


def _frames(n, h, w, seed=0):
    from vdmi import synth
    return synth.frames(n, h, w, seed=seed)


def _rel(a, b):
    return np.abs(a - b).max() / (np.abs(b).max() + 1e-12)


# 16-bit heads vs the f32 oracle: ~1.5x the largest error observed over 1080p / 720p /
# 4K frames and two seeds (tools/observed_tolerances.py on the GPU box: bf16 R50
# <= 0.0116 loc/conf, MobileNet-0.25 <= 0.0273; fp16 R50 <= 0.0018, MobileNet <= 0.0042)
BF16_TOL = {"default": 2e-2, "mnet": 4.5e-2}
FP16_TOL = {"default": 3e-3, "mnet": 6.5e-3}


@pytest.mark.parametrize("wkind", ["default", "mnet"])
def test_heads_bf16_close(gpu, face_ctx_factory, wkind):
    ctx = face_ctx_factory("bf16", 8, wkind)
    fr = _frames(2, 1080, 1920)
    loc, conf, _ = ctx.forward_heads(fr)
    eloc, econf, _ = _oracle_heads(fr, wkind)
    tol = BF16_TOL[wkind]
    assert _rel(loc, eloc) < tol and _rel(conf, econf) < tol


@pytest.mark.parametrize("h,w,wkind", [(1080, 1920, "default"), (2160, 3840, "default"), (1080, 1920, "mnet")])
def test_heads_fp16_close(gpu, face_ctx_factory, h, w, wkind):
    """fp16 mode (VD_PREC_FP16: fp16 operands and activations on
    v_mfma_f32_16x16x32_f16, f32 accumulation; BASELINE config 5 names the fp16
    conv path, here with 4K frames): 10 mantissa bits against bf16's 7, so the
    heads sit an order of magnitude closer to the f32 oracle than bf16's."""
    ctx = face_ctx_factory("fp16", 2, wkind)
    fr = _frames(2, h, w, seed=17)
    loc, conf, ldm = ctx.forward_heads(fr)
    eloc, econf, eldm = _oracle_heads(fr, wkind)
    tol = FP16_TOL[wkind]
    assert _rel(loc, eloc) < tol and _rel(conf, econf) < tol and _rel(ldm, eldm) < tol


def test_detect_fp16_agrees_4k(gpu, face_ctx_factory):
    """fp16 detect + box correction on 4K frames against the f32 oracle's boxes. The
    4K frames are 2x nearest upsamples of 1080p synthetic frames, so the ratio-6
    letterbox (0.5/0.5 bilinear of rows/cols 6x+2, 6x+3) sees real structure and the
    calibrated random weights fire (raw 4K noise averages out to no faces)."""
    ctx = face_ctx_factory("fp16", 2)
    fr = np.repeat(np.repeat(_frames(2, 1080, 1920, seed=17), 2, axis=1), 2, axis=2)
    got = ctx.detect(fr)
    eloc, econf, _ = _oracle_heads(fr)
    pri = oanchors.get_anchors((640, 640))
    matched = total = 0
    for b in range(2):
        _, boxes, _ = obbox.postprocess_frame(eloc[b], econf[b], pri, 0.5, 0.4)
        e = obbox.correct_and_scale(boxes, 2160, 3840)
        g = got.frame(b)[1]
        total += len(e)
        for r in e:
            if len(g) == 0:
                break
            x1 = np.maximum(r[0], g[:, 0]); y1 = np.maximum(r[1], g[:, 1])
            x2 = np.minimum(r[2], g[:, 2]); y2 = np.minimum(r[3], g[:, 3])
            inter = np.clip(x2 - x1, 0, None) * np.clip(y2 - y1, 0, None)
            iou = inter / ((r[2] - r[0]) * (r[3] - r[1]) + (g[:, 2] - g[:, 0]) * (g[:, 3] - g[:, 1]) - inter)
            matched += iou.max() >= 0.9
    assert total > 0 and matched / total >= 0.95, (matched, total)


@pytest.mark.parametrize("prec", ["bf16", "fp16"])
def test_heads_16bit_fused_downsample_matches_unfused(gpu, prec):
    """16-bit plans (bf16; fp16, VD_PREC_FP16, on the same kernels) fuse each bottleneck's conv3 + downsample into one streaming pass
    (layer1.0, layer2.0); option conv_dual=0 at weight load keeps them separate. The
    only numeric difference is the bf16 rounding of the downsample output that the
    unfused plan stores, so the heads agree far tighter than the oracle bound."""
    import vdmi
    fr = _frames(2, 1080, 1920, seed=3)
    out = {}
    for dual in ("1", "0"):
        ctx = vdmi.Context(precision=prec, max_batch=2, options={"conv_dual": int(dual)})
        try:
            ctx.load_weights(0, face_weights("default"))
            out[dual] = ctx.forward_heads(fr)
        finally:
            ctx.close()
    for a, b in zip(out["1"], out["0"]):
        assert _rel(a, b) < (2e-2 if prec == "bf16" else 3e-3)


@pytest.mark.parametrize("prec", ["bf16", "fp16"])
def test_heads_16bit_fused_block_matches_unfused(gpu, prec):
    """bf16 plans run each layer1 bottleneck as one kernel (block.hip: t1/t2 in LDS);
    option block_fuse=0 at weight load keeps the conv-by-conv chain. Same bf16 weights
    and the same bf16 rounding points, only the f32 summation order differs."""
    import vdmi
    fr = _frames(2, 1080, 1920, seed=5)
    out = {}
    for fuse in ("1", "0"):
        ctx = vdmi.Context(precision=prec, max_batch=2, options={"block_fuse": int(fuse)})
        try:
            ctx.load_weights(0, face_weights("default"))
            out[fuse] = ctx.forward_heads(fr)
        finally:
            ctx.close()
    for a, b in zip(out["1"], out["0"]):
        assert _rel(a, b) < (2e-2 if prec == "bf16" else 3e-3)


@pytest.mark.parametrize("prec", ["bf16", "fp16"])
def test_heads_16bit_fused_stem_pool_matches_unfused(gpu, prec):
    """bf16 plans run conv1 + bn1 + relu + maxpool as one kernel (stem.hip: the stem map
    stays in LDS); option stem_pool=0 at weight load keeps the taps conv + maxpool kernels.
    Same products in the same K order and the same bf16 rounding, max pooling is
    exact: the heads are identical."""
    import vdmi
    fr = _frames(2, 720, 1280, seed=9)
    out = {}
    for fuse in ("1", "0"):
        ctx = vdmi.Context(precision=prec, max_batch=2, options={"stem_pool": int(fuse)})
        try:
            ctx.load_weights(0, face_weights("default"))
            out[fuse] = ctx.forward_heads(fr)
        finally:
            ctx.close()
    for a, b in zip(out["1"], out["0"]):
        np.testing.assert_array_equal(a, b)


def test_process_mosaic_exact_given_boxes(gpu, face_ctx_factory):
    """vd_process output == oracle sequential mosaic applied to the GPU's own int boxes."""
    for prec in ("fp32", "bf16"):
        ctx = face_ctx_factory(prec, 8)
        fr = _frames(2, 1080, 1920, seed=4)
        out, faces, _ = ctx.process(fr)
        for b in range(2):
            xi = faces.frame(b)[0]
            exp = omosaic.mosaic_frame(fr[b], [tuple(int(v) for v in r) for r in xi], 8)
            np.testing.assert_array_equal(out[b], exp)
        assert int(faces.count.sum()) > 0


@pytest.mark.parametrize("wkind", ["default", "mnet"])
def test_detect_bf16_agrees(gpu, face_ctx_factory, wkind):
    ctx = face_ctx_factory("bf16", 8, wkind)
    fr = _frames(2, 1080, 1920)
    got = ctx.detect(fr)
    eloc, econf, _ = _oracle_heads(fr, wkind)
    pri = oanchors.get_anchors((640, 640))
    matched = total = 0
    for b in range(2):
        _, boxes, _ = obbox.postprocess_frame(eloc[b], econf[b], pri, 0.5, 0.4)
        e = obbox.correct_and_scale(boxes, 1080, 1920)
        g = got.frame(b)[1]
        total += len(e)
        for r in e:
            if len(g) == 0:
                break
            x1 = np.maximum(r[0], g[:, 0]); y1 = np.maximum(r[1], g[:, 1])
            x2 = np.minimum(r[2], g[:, 2]); y2 = np.minimum(r[3], g[:, 3])
            inter = np.clip(x2 - x1, 0, None) * np.clip(y2 - y1, 0, None)
            iou = inter / ((r[2] - r[0]) * (r[3] - r[1]) + (g[:, 2] - g[:, 0]) * (g[:, 3] - g[:, 1]) - inter)
            matched += iou.max() >= 0.9
    assert total > 0 and matched / total >= 0.9, (matched, total)


def test_retinaface_drop_in(gpu):
    from vdmi import Retinaface
    det = Retinaface(model_path="/nonexistent.pth", backbone="resnet50", input_shape=[640, 640, 3],
                     confidence=0.5, nms_iou=0.4, letterbox_image=True, cuda=True, precision="fp32",
                     max_batch=4, weights=face_weights())
    imgs = list(_frames(3, 720, 1280, seed=9)) + [_frames(1, 1080, 1920, seed=9)[0]]
    res = det.detect_images(imgs)
    assert len(res) == 4
    for (img, boxes), src in zip(res, imgs):
        assert img is src
        assert isinstance(boxes, list) and all(len(b) == 4 and isinstance(b[0], float) for b in boxes)
    # int() of the returned floats == the library's int boxes
    raw = det.detect_boxes(imgs)
    for (_, boxes), (xf, xi, _) in zip(res, raw):
        assert [[int(v) for v in b] for b in boxes] == xi.tolist()


def test_retinaface_drop_in_mobilenet(gpu):
    """Retinaface(backbone="mobilenet") (face.py:35) on seeded random cfg_mnet weights."""
    from vdmi import Retinaface
    det = Retinaface(model_path="/nonexistent.pth", backbone="mobilenet", input_shape=[640, 640, 3],
                     nms_iou=0.4, precision="fp32", max_batch=4, weights=face_weights("mnet"))
    imgs = list(_frames(2, 720, 1280, seed=9))
    res = det.detect_images(imgs)
    assert len(res) == 2 and sum(len(b) for _, b in res) > 0
    raw = det.detect_boxes(imgs)
    for (_, boxes), (xf, xi, _) in zip(res, raw):
        assert [[int(v) for v in b] for b in boxes] == xi.tolist()


@pytest.mark.parametrize("prec", ["bf16", "fp16"])
def test_heads_16bit_chain_matches_unfused(gpu, prec):
    """bf16 plans run layer2's conv3(+bn3+identity+relu) and the next block's conv1
    (+bn1+relu) as one kernel (chain.hip: the block output is handed over in LDS as
    MFMA B fragments); option chain=0 keeps the two streaming launches. Same bf16 weights,
    same K order and the same bf16 rounding points."""
    import vdmi
    fr = _frames(2, 1080, 1920, seed=11)
    out = {}
    for chain in ("1", "0"):
        ctx = vdmi.Context(precision=prec, max_batch=2, options={"chain": int(chain)})
        try:
            ctx.load_weights(0, face_weights("default"))
            out[chain] = ctx.forward_heads(fr)
        finally:
            ctx.close()
    for a, b in zip(out["1"], out["0"]):
        assert _rel(a, b) < (2e-3 if prec == "bf16" else 3e-4), _rel(a, b)


@pytest.mark.parametrize("prec", ["bf16", "fp16"])
def test_heads_16bit_ssh_fused_matches_unfused(gpu, prec):
    """ReLU-SSH plans (cfg_re50) run conv5X5_1 and conv3X3 as one conv with Cout
    64 + 128 on a 192-wide tile, writing [t5 | c3] of one concat buffer (ssh_fuse=1);
    option ssh_fuse=0 keeps the two convs. Every output channel sees the same K order
    and the same rounding: the heads are identical. ssh_fuse=2 (default) fuses
    conv5X5_2 + conv7X7_2 too: heads within accumulation rounding."""
    import vdmi
    fr = _frames(2, 1080, 1920, seed=13)
    out = {}
    for fuse in ("2", "1", "0"):     # 2 (default): conv5X5_2 + conv7X7_2 fused too ([t5|c3|c7|c5|t7])
        ctx = vdmi.Context(precision=prec, max_batch=2, options={"ssh_fuse": int(fuse)})
        try:
            ctx.load_weights(0, face_weights("default"))
            out[fuse] = ctx.forward_heads(fr)
        finally:
            ctx.close()
    for a, b in zip(out["1"], out["0"]):
        np.testing.assert_array_equal(a, b)
    # ssh_fuse=2 also runs conv5X5_2 + conv7X7_2 as one 128-wide conv: another tile form
    # (another in-tile K order) than the two 64-wide convs -- within f32 accumulation
    # rounding of the 16-bit plan, not bit-identical (measured max |diff| ~1e-6)
    for a, b in zip(out["2"], out["0"]):
        assert _rel(a, b) < 1e-4, _rel(a, b)


def test_heads_fp32_ssh_fuse_levels(gpu):
    """fp32 pair plan: ssh_fuse=2 (default; conv5X5_2 + conv7X7_2 as one conv, so
    conv7x7_3 splits t7 with the concat buffer's per-frame scale) against 1 and 0:
    heads within the f32 head bound of each other, identical keep lists and int boxes."""
    import vdmi
    fr = _frames(3, 1080, 1920, seed=31)
    heads, boxes = {}, {}
    for fuse in (2, 1, 0):
        ctx = vdmi.Context(precision="fp32", max_batch=3, options={"ssh_fuse": fuse})
        try:
            ctx.load_weights(0, face_weights("default"))
            heads[fuse] = ctx.forward_heads(fr)
            r = ctx.detect(fr)
            boxes[fuse] = [(r.frame(b)[3].copy(), r.frame(b)[0].copy()) for b in range(3)]
        finally:
            ctx.close()
    assert sum(len(x[0]) for x in boxes[0]) > 0
    for f in (2, 1):
        for a, b in zip(heads[f], heads[0]):
            assert np.abs(a - b).max() <= 6e-6 * (np.abs(b).max() + 1e-6), (f, np.abs(a - b).max())
        for (ka, xa), (kb, xb) in zip(boxes[f], boxes[0]):
            np.testing.assert_array_equal(ka, kb)
            np.testing.assert_array_equal(xa, xb)


def test_heads_fp32_dual_downsample_bit_identical(gpu):
    """fp32 (fp16-pair) plans run layer1.0 / layer2.0's conv3 + downsample as one
    streaming pass (conv1x1_x6_dual_kernel); option conv_dual=0 at weight load stores
    the downsample output and adds it as conv3's residual. Same operand scales, same
    products, the downsample term rounded to f32 before the add in both: the heads
    are bit-identical."""
    import vdmi
    fr = _frames(2, 1080, 1920, seed=13)
    out = {}
    for dual in (1, 0):
        ctx = vdmi.Context(precision="fp32", max_batch=2, options={"conv_dual": dual})
        try:
            ctx.load_weights(0, face_weights("default"))
            out[dual] = ctx.forward_heads(fr)
        finally:
            ctx.close()
    for a, b in zip(out[1], out[0]):
        np.testing.assert_array_equal(a, b)


def test_heads_fp32_exact_canvas_stem_bit_identical(gpu):
    """The face letterbox canvas is integer-valued, exact in fp16: the fp16-pair stem
    then runs with one activation plane and two products (option x6_exact, default
    on). The dropped lo terms are exactly zero, so the heads are bit-identical. (The
    unfused stem: option stem_pool=0; the default fuses stem and pool, below.)"""
    import vdmi
    fr = _frames(2, 720, 1280, seed=19)
    out = {}
    for ex in (1, 0):
        ctx = vdmi.Context(precision="fp32", max_batch=2, options={"x6_exact": ex, "stem_pool": 0})
        try:
            ctx.load_weights(0, face_weights("default"))
            out[ex] = ctx.forward_heads(fr)
        finally:
            ctx.close()
    for a, b in zip(out[1], out[0]):
        np.testing.assert_array_equal(a, b)


def test_heads_fp32_fused_stem_pool_matches_unfused(gpu):
    """fp32 plan, default: conv1 + bn1 + relu + maxpool in one kernel (stem.hip
    stem_pool32_kernel) over an fp16 space-to-depth canvas, the pair weights'
    two products per MAC, f32 stem tile in LDS, f32 pooled map with its per-frame
    max. Against the unfused stem (option stem_pool=0: 7x7 conv on the f32 canvas,
    then maxpool): the same products summed in another order -- heads within f32
    rounding, identical keep lists and boxes."""
    import vdmi
    fr = _frames(3, 1080, 1920, seed=23)
    heads, boxes = {}, {}
    for sp in (1, 0):
        ctx = vdmi.Context(precision="fp32", max_batch=3, options={"stem_pool": sp})
        try:
            ctx.load_weights(0, face_weights("default"))
            heads[sp] = ctx.forward_heads(fr)
            r = ctx.detect(fr)
            boxes[sp] = [r.frame(b)[0].copy() for b in range(3)]
        finally:
            ctx.close()
    for a, b in zip(heads[1], heads[0]):
        assert np.abs(a - b).max() <= 2e-5 * (np.abs(b).max() + 1e-6)
    assert sum(len(x) for x in boxes[0]) > 0
    for a, b in zip(boxes[1], boxes[0]):
        np.testing.assert_array_equal(a, b)


def test_heads_fp32_fused_layer1_matches_unfused(gpu):
    """fp32 plan, default: each layer1 bottleneck as one kernel (block32.hip: t1 / t2 in
    LDS as per-tile-scaled fp16 pairs); option block_fuse32=0 keeps the conv-by-conv
    chain (per-frame scales). The same products rounded at different points: heads
    within f32 rounding of each other (the oracle bound), identical boxes."""
    import vdmi
    fr = _frames(3, 1080, 1920, seed=29)
    heads, boxes = {}, {}
    for fz in (1, 0):
        ctx = vdmi.Context(precision="fp32", max_batch=3, options={"block_fuse32": fz})
        try:
            ctx.load_weights(0, face_weights("default"))
            heads[fz] = ctx.forward_heads(fr)
            r = ctx.detect(fr)
            boxes[fz] = [r.frame(b)[0].copy() for b in range(3)]
        finally:
            ctx.close()
    for a, b in zip(heads[1], heads[0]):
        assert np.abs(a - b).max() <= 6e-6 * (np.abs(b).max() + 1e-6), np.abs(a - b).max() / np.abs(b).max()
    assert sum(len(x) for x in boxes[0]) > 0
    for a, b in zip(boxes[1], boxes[0]):
        np.testing.assert_array_equal(a, b)


def test_heads_fp32_block32_pipe_matches_one_group(gpu):
    """layer1.1 / layer1.2 on the producer / consumer block (option block32_pipe=1,
    default: stage 1 + 3 on waves 0-3, stage 2 on waves 4-7, f32 t1 / t2 split by the
    consumer) against the one-group block (0): the same products and operand scales,
    stage 2 summed in one accumulator instead of two K halves -- heads within f32
    rounding, identical keep lists and int boxes."""
    import vdmi
    fr = _frames(4, 1080, 1920, seed=37)
    heads, boxes = {}, {}
    for pipe in (1, 0):
        ctx = vdmi.Context(precision="fp32", max_batch=4, options={"block32_pipe": pipe})
        try:
            ctx.load_weights(0, face_weights("default"))
            heads[pipe] = ctx.forward_heads(fr)
            r = ctx.detect(fr)
            boxes[pipe] = [(r.frame(b)[3].copy(), r.frame(b)[0].copy()) for b in range(4)]
        finally:
            ctx.close()
    for a, b in zip(heads[1], heads[0]):
        assert np.abs(a - b).max() <= 6e-6 * (np.abs(b).max() + 1e-6), np.abs(a - b).max() / np.abs(b).max()
    assert sum(len(x[0]) for x in boxes[0]) > 0
    for (ka, xa), (kb, xb) in zip(boxes[1], boxes[0]):
        np.testing.assert_array_equal(ka, kb)
        np.testing.assert_array_equal(xa, xb)


def test_heads_fp32_x6_one_bit_identical(gpu):
    """conv_x6_kernel's 1x1 A loads at row offset + scalar K offset (option x6_one)
    fetch the same values as the tap-stepping path: heads bit-identical."""
    import vdmi
    fr = _frames(2, 720, 1280, seed=41)
    heads = {}
    for v in (0, 1):
        ctx = vdmi.Context(precision="fp32", max_batch=2, options={"x6_one": v})
        try:
            ctx.load_weights(0, face_weights("default"))
            heads[v] = ctx.forward_heads(fr)
        finally:
            ctx.close()
    for a, b in zip(heads[1], heads[0]):
        np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("xd", [3, 4])
def test_heads_fp32_block32_depth_bit_identical(gpu, xd):
    """block32.hip's stage-1 x register sets (option block32_xd) only move when the
    loads are issued: heads bit-identical to the default depth."""
    import vdmi
    fr = _frames(2, 720, 1280, seed=31)
    heads = {}
    for d in (2, xd):
        ctx = vdmi.Context(precision="fp32", max_batch=2, options={"block32_xd": d})
        try:
            ctx.load_weights(0, face_weights("default"))
            heads[d] = ctx.forward_heads(fr)
        finally:
            ctx.close()
    for a, b in zip(heads[xd], heads[2]):
        np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("chain,gpw", [(2, 1), (1, 1), (2, 2)])
def test_heads_fp32_chain_matches_unfused(gpu, chain, gpw):
    """fp32 plan, default: layer2's conv3 (+bn3 + identity + relu) and the next block's
    conv1 (+bn1 + relu) as one kernel (chain32.hip: the block output goes to HBM once
    and reaches conv1 from registers, split per (pixel, 64-channel chunk)); option
    chain=0 keeps the two launches (per-frame split). The block outputs are the same;
    conv1's products are rounded at other points: heads within f32 rounding of each
    other, identical boxes. chain=2 (default): layer2's three pairs; chain=1 also layer3's
    five (chain32.hip's 256 -> 1024 -> 256 shape)."""
    import vdmi
    fr = _frames(3, 1080, 1920, seed=37)
    heads, boxes = {}, {}
    for ch in (chain, 0):
        ctx = vdmi.Context(precision="fp32", max_batch=3, options={"chain": ch, "chain_gpw": gpw})
        try:
            ctx.load_weights(0, face_weights("default"))
            heads[ch] = ctx.forward_heads(fr)
            r = ctx.detect(fr)
            boxes[ch] = [r.frame(b)[0].copy() for b in range(3)]
        finally:
            ctx.close()
    for a, b in zip(heads[chain], heads[0]):
        assert np.abs(a - b).max() <= 6e-6 * (np.abs(b).max() + 1e-6), np.abs(a - b).max() / np.abs(b).max()
    assert sum(len(x) for x in boxes[0]) > 0
    for a, b in zip(boxes[chain], boxes[0]):
        np.testing.assert_array_equal(a, b)


def test_heads_fp32_tail_split_bit_identical(gpu):
    """fp32 plan: the big-tile layers' last partial round runs as a second launch of a
    narrower tile (conv_x6.hip launch_x6_big, option x6_tail). The split is along N
    only, so every output keeps its K order and MFMA form: heads bit-identical to the
    unsplit launches. x6_slots=8 makes every big-tile layer of a 3-frame batch split."""
    import vdmi
    fr = _frames(3, 1080, 1920, seed=31)
    heads = {}
    for tail in (0, 1, 2):
        ctx = vdmi.Context(precision="fp32", max_batch=3, options={"x6_tail": tail, "x6_slots": 8})
        try:
            ctx.load_weights(0, face_weights("default"))
            heads[tail] = ctx.forward_heads(fr)
        finally:
            ctx.close()
    for t in (1, 2):
        for a, b in zip(heads[t], heads[0]):
            np.testing.assert_array_equal(a, b)


def test_heads_fp32_halo_tr_bit_identical(gpu):
    """fp32 plan: the halo 3x3 tiles with the MFMA operands exchanged (D^T accumulators,
    weight rows permuted in the DMA, register epilogue; option x6_halo_tr, 1 = the
    128 / 192 / 256-wide tiles, 2 = the narrow 32 / 64-wide ones too) against the
    LDS-staged epilogue (0): the same products in the same order, heads bit-identical."""
    import vdmi
    fr = _frames(2, 1080, 1920, seed=41)
    heads = {}
    for tr in (0, 1, 2):
        ctx = vdmi.Context(precision="fp32", max_batch=2, options={"x6_halo_tr": tr})
        try:
            ctx.load_weights(0, face_weights("default"))
            heads[tr] = ctx.forward_heads(fr)
        finally:
            ctx.close()
    for t in (1, 2):
        for a, b in zip(heads[t], heads[0]):
            np.testing.assert_array_equal(a, b)


def test_heads_fp32_pipelined_b_reads_bit_identical(gpu):
    """fp32 plan, round 6: the halo and wide GEMM tiles read the B fragments of column
    block j + 1 before block j's MFMAs (options x6_halo_pf / x6_gemm_pf, default 1) and
    issue the DMA two K steps ahead between MFMA groups (x6_halo_dma: 0 after the
    barrier, 1 after the MFMAs, 2 between groups, default); the streaming 1x1 layers
    with a residual load it beside the MFMAs (x6_stream_rl, default 1); the 1x1 GEMM
    loop issues the same loads every K tile with one barrier per tile (x6_gemm_uni 2,
    default; 1 keeps two barriers). Schedule only:
    the same products in the same order, heads bit-identical to the round-5 schedule."""
    import vdmi
    fr = _frames(2, 1080, 1920, seed=43)
    heads = {}
    for key, opts in (("r5", {"x6_halo_pf": 0, "x6_gemm_pf": 0, "x6_halo_dma": 0, "x6_stream_rl": 0,
                              "x6_gemm_uni": 0}), ("pf", {}),
                      ("d1", {"x6_halo_dma": 1}), ("u1", {"x6_gemm_uni": 1})):
        ctx = vdmi.Context(precision="fp32", max_batch=2, options=opts)
        try:
            ctx.load_weights(0, face_weights("default"))
            heads[key] = ctx.forward_heads(fr)
        finally:
            ctx.close()
    for k in ("pf", "d1", "u1"):
        for a, b in zip(heads[k], heads["r5"]):
            np.testing.assert_array_equal(a, b)


def test_heads_fp32_halo_conv(gpu):
    """fp32 plan: the 3x3 stride-1 convs with W <= 126 (layer2-4 conv2, FPN merges, SSH
    conv5X5_1 + conv3X3 at levels 0-2) run on conv_x6_halo_kernel (input split once per
    32-channel chunk over the tile's halo; option x6_halo, 2 = three B stages). Same
    products, K summed chunk-major instead of tap-major: heads within f32 rounding of
    the tap-major kernel, identical boxes; the two- and three-stage forms bit-identical
    (same K order; two stages with one or two barriers per step, option x6_halo_1b); batch-invariant (a frame's heads do not depend on its batch mates,
    so halos that straddle frames read only zero padding)."""
    import vdmi
    fr = _frames(3, 1080, 1920, seed=37)
    heads, boxes = {}, {}
    for h in (2, 1, 0):
        ctx = vdmi.Context(precision="fp32", max_batch=3, options={"x6_halo": h})
        try:
            ctx.load_weights(0, face_weights("default"))
            heads[h] = ctx.forward_heads(fr)
            r = ctx.detect(fr)
            boxes[h] = [r.frame(b)[0].copy() for b in range(3)]
            if h:
                one = ctx.forward_heads(fr[1:2])
                for a, b in zip(one, heads[h]):
                    np.testing.assert_array_equal(a[0], b[1])
        finally:
            ctx.close()
    ctx = vdmi.Context(precision="fp32", max_batch=3, options={"x6_halo": 1, "x6_halo_1b": 0})
    try:   # two B stages with two barriers per step (the round-5 loop; default one)
        ctx.load_weights(0, face_weights("default"))
        heads["1b0"] = ctx.forward_heads(fr)
    finally:
        ctx.close()
    for a, b, c in zip(heads[2], heads[1], heads["1b0"]):
        np.testing.assert_array_equal(a, b)
        np.testing.assert_array_equal(c, b)
    for a, b in zip(heads[1], heads[0]):
        assert np.abs(a - b).max() <= 6e-6 * (np.abs(b).max() + 1e-6), np.abs(a - b).max() / np.abs(b).max()
    assert sum(len(x) for x in boxes[0]) > 0
    for a, b in zip(boxes[1], boxes[0]):
        np.testing.assert_array_equal(a, b)


def test_heads_ssh_side_lane_bit_identical(gpu):
    """Face net on two lanes (option ssh_side, default): SSH + heads of levels 1-2 on a
    second stream beside FPN merge1 and level 0 (runtime.cpp Ctx::face_lanes). Same
    kernels on the same operands, so heads and boxes equal the one-stream order bit for
    bit, in both fp32 and bf16; repeated calls (events reused) stay identical."""
    import vdmi
    fr = _frames(3, 1080, 1920, seed=41)
    for prec in ("fp32", "bf16"):
        heads, boxes = {}, {}
        for side in (1, 0):
            ctx = vdmi.Context(precision=prec, max_batch=3, options={"ssh_side": side})
            try:
                ctx.load_weights(0, face_weights("default"))
                heads[side] = ctx.forward_heads(fr)
                again = ctx.forward_heads(fr)
                for a, b in zip(again, heads[side]):
                    np.testing.assert_array_equal(a, b)
                r = ctx.detect(fr)
                boxes[side] = [r.frame(b)[0].copy() for b in range(3)]
            finally:
                ctx.close()
        for a, b in zip(heads[1], heads[0]):
            np.testing.assert_array_equal(a, b)
        for a, b in zip(boxes[1], boxes[0]):
            np.testing.assert_array_equal(a, b)
