"""Hand-derived known-answer tests pinning the CPU oracle to the reference source.

The reference ships no tests or golden vectors; each KAT below is
derived by reading the cited reference line(s) and computing the answer by hand.
"""
import numpy as np
import pytest

from oracle import anchors, bbox, letterbox, mosaic
from oracle.vdexp import vd_expf

F32 = np.float32


# ---------------- anchors: detect_face/utils/anchors.py:22-41 -----------------
def test_anchor_count_and_corners():
    a = anchors.get_anchors((640, 640))
    assert a.shape == (16800, 4) and a.dtype == np.float32        # 80²·2 + 40²·2 + 20²·2
    np.testing.assert_array_equal(a[0], F32([0.00625, 0.00625, 0.025, 0.025]))   # (0.5*8/640, 16/640)
    np.testing.assert_array_equal(a[1], F32([0.00625, 0.00625, 0.05, 0.05]))     # second min_size 32
    np.testing.assert_array_equal(a[2], F32([0.01875, 0.00625, 0.025, 0.025]))   # j=1 -> cx=(1.5*8)/640
    np.testing.assert_array_equal(a[-1], F32([0.975, 0.975, 0.8, 0.8]))          # (19.5*32/640, 512/640)
    np.testing.assert_array_equal(a[12800], F32([0.0125, 0.0125, 0.1, 0.1]))     # level 1 start
    offs, n = anchors.level_offsets((640, 640))
    assert offs == [0, 12800, 16000] and n == 16800
    assert anchors.get_anchors((1280, 1280)).shape == (67200, 4)                  # face.py:20 default


# ---------------- letterbox: utils/utils.py:8-18, resize [ext] ------------------
def _img(h, w, seed=0):
    return np.random.default_rng(seed).integers(0, 256, (h, w, 3), dtype=np.uint8)


def test_letterbox_geometry_16x9():
    for ih, iw in ((1080, 1920), (720, 1280), (2160, 3840)):
        assert letterbox.letterbox_geometry(ih, iw) == (640, 360, 140, 0)
    assert letterbox.letterbox_geometry(640, 640) == (640, 640, 0, 0)
    assert letterbox.letterbox_geometry(480, 640) == (640, 480, 80, 0)


def test_letterbox_1080p_is_exact_gather():
    img = _img(1080, 1920)
    out = letterbox.letterbox_image(img)
    assert out.dtype == np.float64 and out.shape == (640, 640, 3)
    assert (out[:140] == 128).all() and (out[500:] == 128).all()       # (640-360)//2 = 140
    ys, xs = np.arange(360), np.arange(640)
    np.testing.assert_array_equal(out[140:500], img[3 * ys + 1][:, 3 * xs + 1])   # fx = 3dx+1, weights (1,0)


def test_letterbox_720p_is_area_average():
    img = _img(720, 1280).astype(np.int32)
    out = letterbox.letterbox_image(img.astype(np.uint8))[140:500]
    exp = (img[0::2, 0::2] + img[0::2, 1::2] + img[1::2, 0::2] + img[1::2, 1::2] + 2) >> 2
    np.testing.assert_array_equal(out, exp)


def test_letterbox_4k_is_half_half_bilinear():
    img = _img(2160, 3840).astype(np.int32)
    out = letterbox.letterbox_image(img.astype(np.uint8))[140:500]
    r0, r1 = img[2::6], img[3::6]
    exp = (r0[:, 2::6] + r0[:, 3::6] + r1[:, 2::6] + r1[:, 3::6] + 2) >> 2   # fx = 6dx+2.5 -> 1024/1024
    np.testing.assert_array_equal(out, exp)


def test_letterbox_same_size_is_copy_and_mean():
    img = _img(640, 640)
    x, shapes = letterbox.preprocess([img])
    assert x.shape == (1, 3, 640, 640) and x.dtype == np.float32
    np.testing.assert_array_equal(x[0, 0], img[..., 0].astype(np.float32) - 104)   # RGB order, utils.py:28
    np.testing.assert_array_equal(x[0, 2], img[..., 2].astype(np.float32) - 123)
    np.testing.assert_array_equal(shapes, F32([[640, 640]]))
    pad = letterbox.preprocess([_img(1080, 1920)])[0][0, :, 0, 0]
    np.testing.assert_array_equal(pad, F32([24, 11, 5]))   # 128 - mean


def test_yolo_letterbox_geometry():
    # ultralytics LetterBox(640, auto=True, stride=32) [ext]: 1080p -> 640x384, 12 px pad top
    assert letterbox.yolo_letterbox_geometry(1080, 1920) == (640, 360, 12, 0, 384, 640)
    assert letterbox.yolo_letterbox_geometry(640, 640) == (640, 640, 0, 0, 640, 640)
    x = letterbox.yolo_preprocess([_img(1080, 1920)])
    assert x.shape == (1, 3, 384, 640)
    assert x[0, :, 0, 0].tolist() == [F32(114) / F32(255)] * 3


# ---------------- deterministic exp ---------------------------------------------
def test_vd_expf_close_to_correct_rounding():
    rng = np.random.default_rng(0)
    x = np.concatenate([rng.uniform(-100, 88, 200000), rng.uniform(-2, 2, 200000)]).astype(np.float32)
    got = vd_expf(x)
    ref = np.exp(x.astype(np.float64)).astype(np.float32)     # correctly rounded except ~1e-16 cases
    ulps = np.abs(got.view(np.int32).astype(np.int64) - ref.view(np.int32).astype(np.int64))
    assert ulps.max() <= 1 and (ulps == 0).mean() > 0.9999
    assert vd_expf(F32(0.0)) == 1.0 and vd_expf(F32(200)) == np.inf and vd_expf(F32(-200)) == 0.0


# ---------------- decode: utils_bbox.py:49-59 -----------------------------------
def test_decode_operation_order():
    pri = F32([[0.5, 0.5, 0.1, 0.2]])
    loc = F32([[1.0, -2.0, 0.0, 0.0]])
    b = bbox.decode(loc, pri)
    cx = F32(0.5) + (F32(1.0) * F32(0.1)) * F32(0.1)
    cy = F32(0.5) + (F32(-2.0) * F32(0.1)) * F32(0.2)
    x1 = cx - F32(0.1) / F32(2)
    y1 = cy - F32(0.2) / F32(2)
    np.testing.assert_array_equal(b[0], F32([x1, y1, F32(0.1) + x1, F32(0.2) + y1]))   # x2 = w + x1
    # x2 uses the rounded x1, which can differ from cx + w/2 in the last ulp
    pri = F32([[0.3, 0.7, 0.123456, 0.0777]])
    b = bbox.decode(F32([[0.0, 0.0, 0.0, 0.0]]), pri)
    assert b[0, 2] == F32(0.123456) + (F32(0.3) - F32(0.123456) / F32(2))


def test_softmax_score():
    s = bbox.softmax2(F32([[0.0, 0.0], [0.0, 100.0], [3.0, 1.0]]))
    assert s[0, 1] == 0.5 and s[1, 1] == 1.0
    e = vd_expf(F32(-2.0))
    assert s[2, 1] == e / (F32(1.0) + e)


# ---------------- NMS: torchvision nms semantics [ext] ----------------------------
def test_nms_iou_exactly_threshold_is_kept():
    # IoU = 0.5 exactly (representable): [0,0,10,10] vs [0,0,10,5]: inter 50, union 100
    boxes = F32([[0, 0, 10, 10], [0, 0, 10, 5]])
    assert bbox.nms_torchvision(boxes, F32([0.9, 0.8]), 0.5).tolist() == [0, 1]   # suppress only if IoU > thr
    assert bbox.nms_torchvision(boxes, F32([0.9, 0.8]), 0.49).tolist() == [0]


def test_nms_float_ratio_vs_double_threshold():
    # IoU 40/100 in float32 is float32(0.4) = 0.4000000059604645 > 0.4 (the double threshold of
    # combine_detect.py:862) -> suppressed; a float32 compare would have kept it.
    boxes = F32([[0, 0, 10, 10], [0, 0, 10, 4]])
    assert bbox.nms_torchvision(boxes, F32([0.9, 0.8]), 0.4).tolist() == [0]
    boxes = F32([[0, 0, 5, 1], [0, 0, 2, 1]])              # inter 2, union 5 -> float32(0.4) again
    assert bbox.nms_torchvision(boxes, F32([0.9, 0.8]), 0.4).tolist() == [0]
    boxes = F32([[0, 0, 10, 10], [0, 0, 10, 3.9999995]])   # ratio just below 0.4
    assert bbox.nms_torchvision(boxes, F32([0.9, 0.8]), 0.4).tolist() == [0, 1]


def test_nms_ties_are_stable_and_chains():
    boxes = F32([[0, 0, 10, 10], [20, 20, 30, 30], [1, 1, 11, 11], [40, 40, 50, 50]])
    scores = F32([0.7, 0.9, 0.7, 0.9])
    keep = bbox.nms_torchvision(boxes, scores, 0.4)
    assert keep.tolist() == [1, 3, 0]                      # ties: lower index first; 2 suppressed by 0
    # suppressed boxes do not suppress: A > B (IoU>thr), B > C, A !> C -> keep A, C
    boxes = F32([[0, 0, 10, 10], [5, 0, 15, 10], [10, 0, 20, 10]])
    assert bbox.nms_torchvision(boxes, F32([0.9, 0.8, 0.7]), 0.3).tolist() == [0, 2]


def test_postprocess_threshold_inclusive():
    pri = anchors.get_anchors((640, 640))[:4]
    loc = np.zeros((4, 4), np.float32)
    conf = F32([[0, 0], [0, -1], [0, 1], [2, 0]])          # scores 0.5 (kept: >=), <0.5, >0.5, <0.5
    idx, boxes, sc = bbox.postprocess_frame(loc, conf, pri, 0.5, 0.4)
    assert sorted(idx.tolist()) == [0, 2]


# ---------------- box correction: utils_bbox.py:12-43, face.py:144-145 -----------
def test_correct_factors_1080p():
    off, sc = bbox.correct_factors(1080, 1920)
    assert off.tolist() == [0.0, 0.21875]                   # (640-360)/2/640
    assert sc.tolist() == [1.0, F32(640) / F32(360)]
    b = bbox.correct_and_scale(F32([[0.5, 0.21875, 1.0, 0.78125]]), 1080, 1920)
    np.testing.assert_array_equal(b[0], F32([960, 0, 1920, 1080]))


def test_truncation_toward_zero():
    assert bbox.truncate_boxes(F32([[-3.7, 2.9, 0.5, -0.5]])).tolist() == [[-3, 2, 0, 0]]


# ---------------- mosaic: combine_detect.py:138-161 + resizeNN [ext] ---------------
def test_nn_maps():
    assert mosaic.mosaic_axis_map(7).tolist() == [0] * 7                  # bw<8: sw=1 -> top-left
    assert mosaic.mosaic_axis_map(16).tolist() == [0] * 8 + [8] * 8
    assert mosaic.mosaic_axis_map(20).tolist() == [0] * 10 + [10] * 10    # sw=2, ratio 10
    m = mosaic.mosaic_axis_map(23)                                        # sw=2, ratio 11.5
    assert m.tolist() == [0] * 12 + [11] * 11
    assert mosaic.mosaic_axis_map(1).tolist() == [0]


def test_mosaic_single_clip_and_empty():
    img = _img(20, 30)
    out = mosaic.mosaic_rectangle_region_single(img, -5, -5, 3, 4)      # clipped to [0,3)x[0,4)
    exp = img.copy()
    exp[0:4, 0:3] = img[0, 0]
    np.testing.assert_array_equal(out, exp)
    assert out is not img
    np.testing.assert_array_equal(mosaic.mosaic_rectangle_region_single(img, 10, 10, 10, 15), img)
    np.testing.assert_array_equal(mosaic.mosaic_rectangle_region_single(img, 40, 0, 50, 5), img)


def test_mosaic_sequential_overlap_order_matters():
    img = np.zeros((16, 16, 3), np.uint8)
    img[..., 0] = np.arange(16)[None, :]       # value = column index
    a, b = (0, 0, 8, 8), (4, 0, 12, 8)          # both 8 wide -> sw=1 -> fill with left-top pixel
    ab = mosaic.mosaic_frame(img, [a, b])
    ba = mosaic.mosaic_frame(img, [b, a])
    assert ab[0, 4:12, 0].tolist() == [0] * 8   # b reads a's output at column 4 (= 0)
    assert ba[0, 4:12, 0].tolist() == [0, 0, 0, 0, 4, 4, 4, 4]
    assert ba[0, 0:4, 0].tolist() == [0] * 4


def test_mosaic_frame_equals_per_box_copy_composition():
    """oracle.mosaic.mosaic_frame (one copy, in-place per box) == the reference's
    composition of mosaic_rectangle_region_single calls (a fresh array per box,
    combine_detect.py:246-249), incl. overlaps, clipping and empty boxes."""
    from oracle import mosaic as om
    from vdmi import synth
    img = synth.frames(1, 97, 131, seed=5)[0]
    boxes = [tuple(int(v) for v in b) for b in synth.box_lists(1, 97, 131, per_frame=24, seed=9)[0]]
    boxes += [(-5, -5, 7, 40), (120, 90, 200, 200), (30, 30, 30, 60), (10, 10, 14, 13)]
    exp = img.copy()
    for b in boxes:
        exp = om.mosaic_rectangle_region_single(exp, *b, 8)
    np.testing.assert_array_equal(om.mosaic_frame(img, boxes, 8), exp)
    np.testing.assert_array_equal(om.mosaic_frame(img, boxes, 3), _compose(om, img, boxes, 3))


def _compose(om, img, boxes, level):
    out = img.copy()
    for b in boxes:
        out = om.mosaic_rectangle_region_single(out, *b, level)
    return out
