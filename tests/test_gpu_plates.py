"""YOLOv8n plate path (ultralytics semantics, PARITY UNPINNED vs the real
ultralytics — see oracle/yolov8.py) against the CPU oracle:
* fp32 raw Detect outputs within 1e-4 relative of torch-CPU;
* post-processing bit-exact given the same raw outputs (decode, sigmoid, class
  offset NMS, max_det, scale_boxes, clip);
* vd_process with plates mosaicked ("intended mode") equals the oracle's
  sequential mosaic of face boxes then plate boxes (combine_detect.py:242-249)."""
import numpy as np
import pytest
import torch

from oracle import letterbox as olb
from oracle import mosaic as omosaic
from oracle.yolov8 import build_oracle_yolo, postprocess, raw_heads

pytestmark = pytest.mark.gpu

_CTX = {}


def _ctx(precision):
    """precision 'fp32-x6': the fp32 plan on the exact 3-term bf16 split (option f32_split=1)."""
    import vdmi
    from vdmi import weights
    if precision not in _CTX:
        opts = {"f32_split": 1} if precision == "fp32-x6" else {}
        c = vdmi.Context(precision=precision.replace("-x6", ""), max_batch=4, options=opts)
        c.load_weights(0, weights.retinaface_state_dict(0))
        c.load_weights(1, weights.yolov8n_state_dict(0))
        _CTX[precision] = c
    return _CTX[precision]


def _oracle_raw(frames):
    from vdmi import weights
    m = build_oracle_yolo(weights.yolov8n_state_dict(0))
    x = olb.yolo_preprocess(list(frames))
    with torch.no_grad():
        lv = m(torch.from_numpy(x))
    return raw_heads(lv), [tuple(t.shape[2:]) for t in lv], x.shape[2:]


def _rel(a, b):
    return np.abs(a - b).max() / (np.abs(b).max() + 1e-12)


@pytest.mark.parametrize("prec", ["fp32", "fp32-x6"])
@pytest.mark.parametrize("h,w", [(1080, 1920), (720, 1280), (640, 640), (480, 640)])
def test_plate_raw_fp32(gpu, h, w, prec):
    from vdmi import synth
    fr = synth.frames(2, h, w, seed=5)
    got = _ctx(prec).plate_raw(fr)
    exp, _, _ = _oracle_raw(fr)
    assert got.shape == exp.shape
    assert _rel(got, exp) < 1e-4


def test_plate_raw_fp16_close(gpu):
    from vdmi import synth
    fr = synth.frames(2, 1080, 1920, seed=5)
    got = _ctx("fp16").plate_raw(fr)
    exp, _, _ = _oracle_raw(fr)
    assert _rel(got[:, 64:], exp[:, 64:]) < 3e-3      # observed 0.0020 (~1.5x)


def test_plate_raw_bf16_close(gpu):
    from vdmi import synth
    fr = synth.frames(2, 1080, 1920, seed=5)
    got = _ctx("bf16").plate_raw(fr)
    exp, _, _ = _oracle_raw(fr)
    assert _rel(got[:, 64:], exp[:, 64:]) < 5.5e-2    # observed 0.036 (~1.5x)


@pytest.mark.parametrize("prec", ["fp32", "fp32-x6", "bf16"])
def test_plate_post_exact_given_raw(gpu, prec):
    from vdmi import synth
    ctx = _ctx(prec)
    fr = synth.frames(3, 1080, 1920, seed=6)
    raw = ctx.plate_raw(fr)
    shapes = [(48, 80), (24, 40), (12, 20)]
    exp = postprocess(raw, shapes, (384, 640), (1080, 1920))
    got = ctx.detect_plates(fr)
    n = 0
    for b in range(3):
        xi, xf, sc, lab = got.frame(b)
        e_xy, e_conf, e_cls, _ = exp[b]
        assert int(got.count[b]) == len(e_xy)
        np.testing.assert_array_equal(xf, e_xy)
        np.testing.assert_array_equal(sc, e_conf)
        np.testing.assert_array_equal(lab, e_cls)
        np.testing.assert_array_equal(xi, np.trunc(e_xy).astype(np.int64))
        n += len(e_xy)
    assert n > 0


def test_yolo_drop_in_results(gpu):
    from vdmi import YOLO, synth
    det = YOLO(weights="random", precision="fp32", max_batch=4).cuda()
    imgs = list(synth.frames(2, 1080, 1920, seed=6))
    res = det(imgs, verbose=False, conf=0.5)
    assert len(res) == 2 and all(r.orig_shape == (1080, 1920) for r in res)
    assert all(r.boxes.xyxy.shape[1] == 4 for r in res)
    assert next(det.model.parameters()).device.type == "cuda"
    # the reference's tuple check (combine_detect.py:239) yields no plate boxes for Results
    assert [r[1] if isinstance(r, tuple) else [] for r in res] == [[], []]


def test_process_faces_and_plates_mosaic(gpu):
    from vdmi import _lib, synth
    ctx = _ctx("bf16")
    fr = synth.frames(2, 1080, 1920, seed=8)
    flags = _lib.VD_PROC_FACES | _lib.VD_PROC_PLATES | _lib.VD_PROC_MOSAIC | _lib.VD_PROC_MOSAIC_PLATES
    out, faces, plates = ctx.process(fr, flags=flags)
    ref_flags = _lib.VD_PROC_FACES | _lib.VD_PROC_PLATES | _lib.VD_PROC_MOSAIC
    out_ref, faces2, _ = ctx.process(fr, flags=ref_flags)
    for b in range(2):
        fb = [tuple(int(v) for v in r) for r in faces.frame(b)[0]]
        pb = [tuple(int(v) for v in r) for r in plates.frame(b)[0]]
        np.testing.assert_array_equal(out[b], omosaic.mosaic_frame(fr[b], fb + pb, 8))
        # reference mode: plate boxes discarded (combine_detect.py:239)
        np.testing.assert_array_equal(out_ref[b], omosaic.mosaic_frame(fr[b], fb, 8))
    assert int(plates.count.sum()) > 0


@pytest.mark.parametrize("h,w", [(1080, 1920), (720, 1280), (640, 640), (480, 640)])
def test_plate_raw_bf16_s2d_matches_plain(gpu, h, w):
    """bf16 plans letterbox the plate canvas in space-to-depth form and run model.0
    (3x3 stride 2) as a 2x2 conv over it (plate_net.cpp yconv_s2d); option plate_s2d=0
    keeps the 8-channel canvas and the 3x3 conv. Same 27 products per output in
    another f32 order: the raw outputs agree to bf16 rounding, and both stay within
    the bf16 oracle bound."""
    import vdmi
    from vdmi import synth, weights
    fr = synth.frames(2, h, w, seed=7)
    out = {}
    for s2d in ("1", "0"):
        c = vdmi.Context(precision="bf16", max_batch=2, options={"plate_s2d": int(s2d)})
        try:
            c.load_weights(1, weights.yolov8n_state_dict(0))
            out[s2d] = c.plate_raw(fr)
        finally:
            c.close()
    exp, _, _ = _oracle_raw(fr)
    assert out["1"].shape == out["0"].shape == exp.shape
    assert _rel(out["1"][:, 64:], out["0"][:, 64:]) < 2e-2
    assert _rel(out["1"][:, 64:], exp[:, 64:]) < 8e-2


@pytest.mark.parametrize("prec,h,w", [("bf16", 1080, 1920), ("bf16", 720, 1280), ("bf16", 480, 640),
                                       ("bf16", 1080, 1440), ("fp32", 1080, 1920), ("fp16", 720, 1280)])
def test_process_paired_letterbox_matches_separate(gpu, prec, h, w):
    """With faces and plates in one vd_process call, both s2d canvases come from one
    read of the frames (pre.hip letterbox_s2d_pair_kernel) where the resize geometry
    matches; option lb_pair=0 runs the two letterboxes apart. Same per-pixel arithmetic
    (fp32 plan: fp16 face canvas + f32 plate canvas from the one staged read): box lists
    and mosaicked frames are identical."""
    import vdmi
    from vdmi import _lib, synth, weights
    fr = synth.frames(2, h, w, seed=21)
    flags = _lib.VD_PROC_FACES | _lib.VD_PROC_PLATES | _lib.VD_PROC_MOSAIC | _lib.VD_PROC_MOSAIC_PLATES
    res = {}
    for pair in ("1", "0"):
        c = vdmi.Context(precision=prec, max_batch=2, options={"lb_pair": int(pair)})
        try:
            c.load_weights(0, weights.retinaface_state_dict(0))
            c.load_weights(1, weights.yolov8n_state_dict(0))
            c.timing(True)
            c.timing_reset()
            out, faces, plates = c.process(fr, flags=flags)
            _, n_lb, _ = c.timing_read(_lib.FAM_LETTERBOX)
            assert n_lb == (1 if pair == "1" else 2), (pair, n_lb)   # the paired kernel really ran
            res[pair] = (out.copy(), [faces.frame(b)[0].copy() for b in range(2)],
                         [plates.frame(b)[0].copy() for b in range(2)])
        finally:
            c.close()
    np.testing.assert_array_equal(res["1"][0], res["0"][0])
    assert sum(len(x) for x in res["1"][1] + res["1"][2]) > 0      # boxes were found to compare
    for b in range(2):
        np.testing.assert_array_equal(res["1"][1][b], res["0"][1][b])
        np.testing.assert_array_equal(res["1"][2][b], res["0"][2][b])


@pytest.mark.parametrize("stage", [0, 1, 5])
def test_process_plate_release_point(gpu, stage):
    """Option plate_stage holds the plate branch back until face stage N has been
    issued (default 3: its HBM-bound convs then overlap the MFMA-bound late face
    layers). Scheduling only: the fp32 boxes and mosaicked frames equal the default's."""
    import vdmi
    from vdmi import _lib, synth, weights
    fr = synth.frames(3, 1080, 1920, seed=22)
    flags = _lib.VD_PROC_FACES | _lib.VD_PROC_PLATES | _lib.VD_PROC_MOSAIC | _lib.VD_PROC_MOSAIC_PLATES
    res = {}
    for st in (stage, 3):
        c = vdmi.Context(precision="fp32", max_batch=3, options={"plate_stage": st})
        try:
            c.load_weights(0, weights.retinaface_state_dict(0))
            c.load_weights(1, weights.yolov8n_state_dict(0))
            for _ in range(2):                                     # a second call reuses the event
                out, faces, plates = c.process(fr, flags=flags)
            res[st] = (out.copy(), [faces.frame(b)[0].copy() for b in range(3)],
                       [plates.frame(b)[0].copy() for b in range(3)])
        finally:
            c.close()
    np.testing.assert_array_equal(res[stage][0], res[3][0])
    assert sum(len(x) for x in res[3][1] + res[3][2]) > 0
    for b in range(3):
        np.testing.assert_array_equal(res[stage][1][b], res[3][1][b])
        np.testing.assert_array_equal(res[stage][2][b], res[3][2][b])


@pytest.mark.parametrize("mosaic_plates", [False, True])
def test_process_detect_early_and_mosaic_early_identical(gpu, mosaic_plates):
    """Round 6 scheduling options: plate_detect_early (each YOLO Detect level right after
    its P level; default 1) and mosaic_early (without MOSAIC_PLATES the face mosaic runs
    before the plate branch joins; default 1). Order only: the plate raw heads, both box
    lists and the mosaicked frames equal the all-at-the-end schedule's, in both plate modes
    (combine_detect.py:239 discards plate boxes; the intended mode blurs them)."""
    import vdmi
    from vdmi import _lib, synth, weights
    fr = synth.frames(3, 1080, 1920, seed=23)
    flags = _lib.VD_PROC_FACES | _lib.VD_PROC_PLATES | _lib.VD_PROC_MOSAIC
    if mosaic_plates:
        flags |= _lib.VD_PROC_MOSAIC_PLATES
    res = {}
    for key, opts in (("new", {}), ("old", {"plate_detect_early": 0, "mosaic_early": 0})):
        c = vdmi.Context(precision="fp32", max_batch=3, options=opts)
        try:
            c.load_weights(0, weights.retinaface_state_dict(0))
            c.load_weights(1, weights.yolov8n_state_dict(0))
            raw = c.plate_raw(fr)
            for _ in range(2):
                out, faces, plates = c.process(fr, flags=flags)
            res[key] = (raw, out.copy(), [faces.frame(b)[0].copy() for b in range(3)],
                        [plates.frame(b)[0].copy() for b in range(3)])
        finally:
            c.close()
    np.testing.assert_array_equal(res["new"][0], res["old"][0])
    np.testing.assert_array_equal(res["new"][1], res["old"][1])
    assert sum(len(x) for x in res["old"][2]) > 0
    for b in range(3):
        np.testing.assert_array_equal(res["new"][2][b], res["old"][2][b])
        np.testing.assert_array_equal(res["new"][3][b], res["old"][3][b])


@pytest.mark.parametrize("prec,plates,groups", [("fp32", True, 2), ("fp32", False, 2), ("bf16", True, 2),
                                               ("fp32", True, 3), ("fp16", False, 4)])
def test_process_face_groups_bit_identical(gpu, prec, plates, groups):
    """Option face_groups runs the face net as G frame groups on G streams (runtime.cpp
    Ctx::face_forward; default 2). Every kernel is batch-invariant, so the float boxes,
    scores and mosaicked frames equal the one-launch schedule's (face_groups=1)
    exactly; an odd batch splits unevenly (5 frames: 2 + 3, 1 + 2 + 2, 1 + 1 + 1 + 2)."""
    import vdmi
    from vdmi import _lib, synth, weights
    fr = synth.frames(5, 1080, 1920, seed=23)
    flags = _lib.VD_PROC_FACES | _lib.VD_PROC_MOSAIC
    if plates:
        flags |= _lib.VD_PROC_PLATES | _lib.VD_PROC_MOSAIC_PLATES
    res = {}
    for hv in (groups, 1):
        c = vdmi.Context(precision=prec, max_batch=5, options={"face_groups": hv})
        try:
            c.load_weights(0, weights.retinaface_state_dict(0))
            if plates:
                c.load_weights(1, weights.yolov8n_state_dict(0))
            for _ in range(2):                                     # a second call reuses the events
                out, faces, pl = c.process(fr, flags=flags)
            res[hv] = (out.copy(), [faces.frame(b)[0].copy() for b in range(5)],
                       [np.concatenate([faces.frame(b)[1].ravel(), faces.frame(b)[2]]) for b in range(5)])
        finally:
            c.close()
    np.testing.assert_array_equal(res[groups][0], res[1][0])
    assert sum(len(x) for x in res[1][1]) > 0
    for b in range(5):
        np.testing.assert_array_equal(res[groups][1][b], res[1][1][b])
        np.testing.assert_array_equal(res[groups][2][b], res[1][2][b])


@pytest.mark.parametrize("h,w", [(1080, 1920), (720, 1280), (480, 640)])
def test_plate_raw_fp32_s2d_matches_plain(gpu, h, w):
    """fp32 plan: the plate canvas in space-to-depth form as integer pixel values in
    fp16 (exact), model.0 as a 2x2 conv over it on one A plane with the / 255 folded
    into its BN scale (plate_net.cpp yconv_s2d, option plate_s2d32); plate_s2d32=0
    keeps the f32 canvas and the 3x3 conv. The same 27 products per output in another
    f32 order: raw outputs within f32 rounding of each other and of the oracle."""
    import vdmi
    from vdmi import synth, weights
    fr = synth.frames(2, h, w, seed=7)
    out = {}
    for s2d in (1, 0):
        c = vdmi.Context(precision="fp32", max_batch=2, options={"plate_s2d32": s2d})
        try:
            c.load_weights(1, weights.yolov8n_state_dict(0))
            out[s2d] = c.plate_raw(fr)
        finally:
            c.close()
    exp, _, _ = _oracle_raw(fr)
    assert out[1].shape == out[0].shape == exp.shape
    assert _rel(out[1], out[0]) < 2e-5
    assert _rel(out[1], exp) < 1e-4


@pytest.mark.parametrize("h,w", [(1080, 1920), (720, 1280), (480, 640)])
def test_plate_raw_fp32_taps_matches_gemm(gpu, h, w):
    """fp32 plan: the YOLO net's narrow KxK layers (model.0 on its integer s2d canvas,
    model.1 / model.3 and the C2f bottleneck 3x3 convs with K <= 288) on the streaming
    TAPS form (conv_x6.hip conv1x1_x6_kernel<..., TAPS>, option x6_taps); x6_taps=0 runs
    them on the GEMM / halo tiles. The same fp16-pair products per output in another f32
    order: raw outputs within f32 rounding of each other and of the oracle, the same
    int boxes, float corners within f32 rounding."""
    import vdmi
    from vdmi import synth, weights
    fr = synth.frames(3, h, w, seed=9)
    out, boxes = {}, {}
    for t in (1, 0):
        c = vdmi.Context(precision="fp32", max_batch=3, options={"x6_taps": t})
        try:
            c.load_weights(1, weights.yolov8n_state_dict(0))
            c.timing(True)
            c.timing_reset()
            out[t] = c.plate_raw(fr)
            got = c.detect_plates(fr)
            boxes[t] = [(got.frame(b)[0].copy(), got.frame(b)[1].copy()) for b in range(3)]
        finally:
            c.close()
    exp, _, _ = _oracle_raw(fr)
    assert out[1].shape == out[0].shape == exp.shape
    assert _rel(out[1], out[0]) < 2e-5
    assert _rel(out[1], exp) < 1e-4
    for b in range(3):   # same boxes; float corners within f32 rounding (observed 2e-7)
        np.testing.assert_array_equal(boxes[1][b][0], boxes[0][b][0])
        np.testing.assert_allclose(boxes[1][b][1], boxes[0][b][1], rtol=2e-6, atol=0)


@pytest.mark.parametrize("h,w", [(1080, 1920), (480, 640)])
def test_plate_raw_fp32_grouped_det_bit_identical(gpu, h, w):
    """fp32 plan: the Detect heads' cv2.i.1 and cv3.i.1 (3x3, 64 -> 64 on the two halves
    of det0.i's output) as one grouped conv on the halo tile (option det_group: each
    64-wide N tile reads its group's 64 input channels). The same tile form and K order
    as the two convs (det_group=0): raw outputs bit-identical."""
    import vdmi
    from vdmi import synth, weights
    fr = synth.frames(2, h, w, seed=47)
    out = {}
    for g in (1, 0):
        c = vdmi.Context(precision="fp32", max_batch=2, options={"det_group": g})
        try:
            c.load_weights(1, weights.yolov8n_state_dict(0))
            out[g] = c.plate_raw(fr)
        finally:
            c.close()
    np.testing.assert_array_equal(out[1], out[0])
