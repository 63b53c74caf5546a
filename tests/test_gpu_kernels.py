"""GPU parity of the individual HIP kernels against the CPU oracle (through the C-ABI).

Bar: bit-exact for integer/byte/index work (mosaic, letterbox, NMS keep lists,
int boxes); the conv kernel against a torch-CPU fp32 conv with the tolerances
written in each test (exact-f32 MFMA mode: 1e-5 relative to the layer's scale;
bf16 mode: 2e-2 relative)."""
import numpy as np
import pytest
import torch

from oracle import anchors as oanchors
from oracle import bbox as obbox
from oracle import letterbox as olb
from oracle import mosaic as omosaic

pytestmark = pytest.mark.gpu
F32 = np.float32


# ------------------------------------------------------------------ mosaic
def _rand_boxes(rng, n, h, w, k):
    out = []
    for _ in range(n):
        bl = []
        for _ in range(k):
            bw, bh = rng.integers(1, max(2, w // 3)), rng.integers(1, max(2, h // 3))
            x1, y1 = rng.integers(-bw, w), rng.integers(-bh, h)
            bl.append((int(x1), int(y1), int(x1 + bw), int(y1 + bh)))
        # degenerate / inverted / fully outside
        bl += [(5, 5, 5, 9), (9, 9, 3, 3), (w + 3, 0, w + 9, 4)]
        rng.shuffle(bl)
        out.append(bl)
    return out


@pytest.mark.parametrize("h,w,k", [(64, 80, 12), (37, 51, 30), (1080, 1920, 16), (720, 1280, 8)])
def test_mosaic_matches_oracle(gpu, face_ctx_factory, h, w, k):
    from vdmi import mosaic_frames, synth
    ctx = face_ctx_factory("bf16", 8)
    rng = np.random.default_rng(h * 1000 + w)
    n = 3
    frames = synth.frames(n, h, w, seed=7)
    boxes = _rand_boxes(rng, n, h, w, k)
    got = mosaic_frames(frames, boxes, 8, ctx=ctx)
    for i in range(n):
        exp = omosaic.mosaic_frame(frames[i], boxes[i], 8)
        np.testing.assert_array_equal(got[i], exp)


@pytest.mark.parametrize("nt", [1, 3])
def test_mosaic_nontemporal_matches_oracle(gpu, nt):
    """Option mosaic_nt: the output pass's stores (1) and source loads (3) non-temporal
    -- the same bytes."""
    import vdmi
    from vdmi import mosaic_frames, synth
    ctx = vdmi.Context(precision="bf16", max_batch=4, options={"mosaic_nt": nt})
    try:
        rng = np.random.default_rng(5)
        frames = synth.frames(3, 1080, 1920, seed=9)
        boxes = _rand_boxes(rng, 3, 1080, 1920, 20)
        got = mosaic_frames(frames, boxes, 8, ctx=ctx)
        for i in range(3):
            np.testing.assert_array_equal(got[i], omosaic.mosaic_frame(frames[i], boxes[i], 8))
    finally:
        ctx.close()


def test_mosaic_nested_chain_and_levels(gpu, face_ctx_factory):
    """Deeply nested boxes force walks that leave a row band (global fallback)."""
    from vdmi import mosaic_frames, synth
    ctx = face_ctx_factory("bf16", 8)
    frames = synth.frames(2, 300, 200, seed=3)
    boxes = [[(10 + 3 * i, 5 + 9 * i, 190 - 2 * i, 295 - i) for i in range(25)],
             [(0, 0, 200, 300), (50, 50, 60, 61), (0, 150, 100, 300), (20, 0, 23, 300)]]
    for level in (2, 8, 16):
        got = mosaic_frames(frames, boxes, level, ctx=ctx)
        for i in range(2):
            np.testing.assert_array_equal(got[i], omosaic.mosaic_frame(frames[i], boxes[i], level))


def test_mosaic_cell_table_overflow(gpu, face_ctx_factory):
    """Level 1 on large boxes: more mosaic cells than the per-frame cell table
    holds (2^18), so the frame takes the per-pixel walk; mixed with a frame that
    uses the table."""
    from vdmi import mosaic_frames, synth
    ctx = face_ctx_factory("bf16", 8)
    frames = synth.frames(2, 480, 720, seed=9)
    boxes = [[(0, 0, 720, 480), (100, 50, 600, 400), (30, 20, 700, 470)],
             [(10, 10, 90, 70), (50, 40, 200, 160)]]
    for level in (1, 3):
        got = mosaic_frames(frames, boxes, level, ctx=ctx)
        for i in range(2):
            np.testing.assert_array_equal(got[i], omosaic.mosaic_frame(frames[i], boxes[i], level))


def test_mosaic_many_boxes_band_overflow(gpu, face_ctx_factory):
    from vdmi import mosaic_frames, synth
    ctx = face_ctx_factory("bf16", 8)
    rng = np.random.default_rng(5)
    frames = synth.frames(1, 96, 128, seed=4)
    boxes = [[tuple(int(v) for v in (x, y, x + rng.integers(1, 30), y + rng.integers(1, 30)))
              for x, y in zip(rng.integers(-10, 128, 600), rng.integers(-10, 96, 600))]]
    got = mosaic_frames(frames, boxes, 8, ctx=ctx)
    np.testing.assert_array_equal(got[0], omosaic.mosaic_frame(frames[0], boxes[0], 8))


@pytest.mark.parametrize("nbox", [255, 256, 257])
def test_mosaic_box_count_boundary(gpu, face_ctx_factory, nbox):
    """Frames at the fast-path box limit (256: overlap graph + cell table; 257:
    per-pixel walk), next to a frame with no boxes and one with a single box."""
    from vdmi import mosaic_frames, synth
    ctx = face_ctx_factory("bf16", 8)
    rng = np.random.default_rng(nbox)
    h, w = 270, 480
    frames = synth.frames(3, h, w, seed=nbox)
    big = [tuple(int(v) for v in (x, y, x + rng.integers(4, 60), y + rng.integers(4, 60)))
           for x, y in zip(rng.integers(-20, w, nbox), rng.integers(-20, h, nbox))]
    boxes = [big, [], [(100, 50, 300, 200)]]
    got = mosaic_frames(frames, boxes, 8, ctx=ctx)
    for i in range(3):
        np.testing.assert_array_equal(got[i], omosaic.mosaic_frame(frames[i], boxes[i], 8))


def test_mosaic_wide_band_arena_overflow(gpu, face_ctx_factory):
    """Bands whose boxes' widths sum past the per-band column map (3072 columns)
    compute the cell column per pixel, bands whose cells exceed the LDS slice
    (2048) read the global cell table; mixed with bands that fit."""
    from vdmi import mosaic_frames, synth
    ctx = face_ctx_factory("bf16", 8)
    frames = synth.frames(3, 1080, 1920, seed=11)
    boxes = [[(17 * i, 100 + 9 * i, 1900 - 13 * i, 400 + 7 * i) for i in range(12)] + [(5, 700, 333, 1000)],
             [(0, 0, 1920, 1080), (100, 100, 1800, 1000), (3, 5, 1917, 1077), (600, 0, 1300, 1080)],
             [(100, 200, 1100, 600), (900, 500, 1500, 900)]]   # level 2: cells overflow the LDS slice
    for level in (2, 5, 8):
        got = mosaic_frames(frames, boxes, level, ctx=ctx)
        for i in range(3):
            np.testing.assert_array_equal(got[i], omosaic.mosaic_frame(frames[i], boxes[i], level))


def test_mosaic_row_classes_and_wide_cells(gpu, face_ctx_factory):
    """Bands with more distinct row box-sets than column maps (staggered box tops
    inside one band), and a level-1 box wider than the map's 11-bit cell column."""
    from vdmi import mosaic_frames, synth
    ctx = face_ctx_factory("bf16", 8)
    frames = synth.frames(2, 1080, 1920, seed=13)
    stag = [(40 + 150 * i, 33 + 2 * i, 200 + 150 * i, 90 + 3 * i) for i in range(12)]
    stag += [(0, 36, 1920, 41), (500, 30, 900, 47)]
    got = mosaic_frames(frames, [stag, stag[::-1]], 8, ctx=ctx)
    for i, bl in enumerate([stag, stag[::-1]]):
        np.testing.assert_array_equal(got[i], omosaic.mosaic_frame(frames[i], bl, 8))
    wide = synth.frames(1, 96, 2208, seed=14)
    bl = [(3, 5, 2150, 60), (100, 20, 300, 90)]
    for level in (1, 2):
        got = mosaic_frames(wide, [bl], level, ctx=ctx)
        np.testing.assert_array_equal(got[0], omosaic.mosaic_frame(wide[0], bl, level))


def test_mosaic_single_drop_in(gpu):
    from vdmi import mosaic_rectangle_region_single, synth
    img = synth.frame(120, 160, 0)
    for box in [(10, 20, 90, 100), (-5, -5, 7, 9), (150, 100, 400, 400), (30, 30, 30, 40)]:
        got = mosaic_rectangle_region_single(img, *box, mosaic_level=8)
        np.testing.assert_array_equal(got, omosaic.mosaic_rectangle_region_single(img, *box, 8))
        assert got is not img


# ------------------------------------------------------------------ letterbox
@pytest.mark.parametrize("prec", ["fp32", "bf16"])
@pytest.mark.parametrize("h,w", [(1080, 1920), (720, 1280), (2160, 3840), (640, 640), (480, 640), (333, 517)])
def test_letterbox_matches_oracle(gpu, face_ctx_factory, prec, h, w):
    from vdmi import synth
    ctx = face_ctx_factory(prec, 8)
    frames = synth.frames(2, h, w, seed=11)
    got = ctx.letterbox(frames, cpad=3)                 # NHWC, 3 real channels
    exp, _ = olb.preprocess(list(frames))               # NCHW
    np.testing.assert_array_equal(got, exp.transpose(0, 2, 3, 1))   # integers: exact in bf16 too


# ------------------------------------------------------------------ conv
CONV_CASES = [
    # (n, h, w, cin, cout, k, stride, pad, act, res_mode)
    (2, 17, 19, 64, 64, 1, 1, 0, 1, 0),
    (2, 17, 19, 64, 128, 3, 1, 1, 1, 0),
    (1, 33, 31, 128, 256, 3, 2, 1, 1, 0),
    (2, 20, 20, 256, 64, 1, 1, 0, 0, 1),
    (1, 40, 36, 3, 64, 7, 2, 3, 1, 0),        # stem, generic tap loader
    (2, 24, 20, 16, 32, 3, 2, 1, 3, 0),       # YOLO-style small C, SiLU
    (1, 16, 16, 48, 24, 1, 1, 0, 3, 2),       # cin 48 generic, res after act
    (1, 12, 10, 256, 32, 1, 1, 0, 0, 0),      # heads (BN=32 tile)
    (1, 9, 11, 512, 200, 3, 1, 1, 2, 1),      # cout not a tile multiple, leaky
    (2, 23, 21, 256, 192, 3, 1, 1, 1, 0),     # 192-wide N tile: fused SSH conv5X5_1 + conv3X3
    (2, 13, 11, 256, 512, 3, 1, 1, 1, 1),     # fp32 pairs: 256 x 256 tile, two N tiles, residual, M tail
    (1, 15, 17, 64, 160, 3, 1, 1, 2, 1),      # 192-wide N tile, cout 160, leaky + residual
    # fp32 halo form (3x3 / stride 1, Cin % 32 == 0, W <= 126): the widest halo, N = 32 / 64
    # tiles, frames smaller than a tile (one tile's halo straddles several frames), W past the limit
    (1, 5, 126, 32, 64, 3, 1, 1, 1, 0),
    (3, 7, 9, 64, 32, 3, 1, 1, 2, 1),
    (2, 6, 127, 32, 128, 3, 1, 1, 1, 0),
    # 1x1 streaming kernel (bf16, K 64/128/256/512): bottleneck conv3 / conv1 / downsample shapes
    (2, 21, 23, 64, 256, 1, 1, 0, 1, 1),      # conv3 + residual, M not a multiple of 16
    (1, 18, 18, 256, 512, 1, 2, 0, 0, 0),     # stride-2 downsample
    (1, 10, 14, 128, 512, 1, 1, 0, 1, 1),
    (2, 9, 7, 256, 128, 1, 1, 0, 3, 0),       # SiLU
    (1, 13, 11, 128, 192, 1, 1, 0, 0, 2),     # residual after (no) activation, 64-channel slices
    # 1x1 streaming kernel at K = 512 (16 k-steps, 128 KB weight slice in LDS)
    (2, 15, 17, 512, 128, 1, 1, 0, 1, 0),     # bottleneck conv1 of layer2
    (1, 18, 18, 512, 256, 1, 2, 0, 0, 0),     # stride-2 downsample (layer3.0)
    (1, 9, 10, 512, 256, 1, 1, 0, 1, 1),      # residual before ReLU (layer4 conv3 form)
    (1, 11, 13, 512, 192, 1, 1, 0, 0, 2),     # 64-channel slices, residual after activation
    # 256-channel slices (K 128/256, Cout % 256 == 0): layer2/3 conv3 + identity
    (2, 10, 13, 128, 512, 1, 1, 0, 1, 1),
    (1, 9, 9, 256, 1024, 1, 1, 0, 1, 1),
    (1, 12, 11, 256, 256, 1, 2, 0, 0, 0),     # stride 2, one chunk
    # streaming taps kernel (K <= 320, Cout % 16 == 0): YOLO C2f bottleneck / 1x1 / stride-2 shapes
    (2, 14, 18, 16, 16, 3, 1, 1, 3, 2),       # 16-channel slice, SiLU, shortcut after activation
    (1, 20, 22, 32, 48, 1, 1, 0, 3, 0),       # 1x1 with K 32 (< one k-tile), three 16-channel slices
    (1, 31, 29, 32, 64, 3, 2, 1, 3, 0),       # stride 2, K 288, odd spatial dims
]


@pytest.mark.parametrize("prec", ["fp32", "fp32-big", "fp32-mf32", "fp32-mid", "fp32-small", "fp32-halo1", "fp32-exact", "fp32-x6",
                                  "fp32-x6-big", "fp32-x6-small", "fp32-s128", "fp32-s256", "bf16", "fp16", "bf16-gemm64",
                                  "bf16-gemm128"])
@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_matches_torch(gpu, face_ctx_factory, prec, case, options=None):
    """fp32: the default fp32 plan (conv_x6.hip, scaled fp16 pairs on the f16 matrix
    cores: streaming 1x1 for K in {64,128,256}, else the tiled GEMM; -big / -small
    force its 256-row two-stage / 128-row one-stage tile; the hook also checks the
    kernel's per-frame output max slots against the host max of the result);
    fp32-exact: exact-f32 MFMA (option f32_split=0); fp32-x6(-big/-small): the exact
    3-term bf16 split (option f32_split=1); bf16: the default dispatch
    (streaming 1x1 / streaming taps / phased / GEMM); bf16-gemm64 / -gemm128: the
    implicit GEMM with 64- and 128-row tiles forced through vd_set_option. The default
    fp32 plan runs the 3x3 stride-1 shapes (Cin % 32 == 0, W <= 126) on the halo form
    (three B stages; fp32-halo1: two); -big / -small / -mf32 switch it off so the
    tap-major tiles keep their coverage on those shapes."""
    options = dict(options or {})
    if prec == "fp32-halo1":
        options.update(x6_halo=1)
        prec = "fp32"
    if prec in ("fp32-big", "fp32-small", "fp32-mf32"):
        options.update(x6_halo=0)
    if prec in ("fp32-s128", "fp32-s256"):     # streaming 1x1 slices of 128 / 256 (default) channels, K 64 / 128
        options.update(x6_stream256=0 if prec == "fp32-s128" else 2)
        prec = "fp32"
    if prec.startswith("fp32-x6"):
        options.update(f32_split=1)
        prec = prec.replace("-x6", "")
    if prec == "fp32-exact":
        options.update(f32_split=0)
        prec = "fp32"
    if prec == "fp32-mid":                    # 1x1 Cout-128 convs on the 128 x 128 two-stage tile (option x6_mid)
        options.update(x6_mid=1 << 20, x6_stream=0)
        prec = "fp32"
    if prec == "fp32-mf32":                   # the big tile on v_mfma_f32_32x32x16_f16 (option x6_mf32)
        options.update(x6_mf32=1)
        prec = "fp32-big"
    if prec in ("fp32-big", "fp32-small"):    # force one x6 tile form (conv_x6.hip)
        options.update(x6_small_k=0, x6_small_k2=0, x6_small_tiles=0, x6_stream=0) if prec == "fp32-big" else \
            options.update(x6_small_k=1 << 30, x6_stream=0)
        prec = "fp32"
    if prec.startswith("bf16-gemm"):
        options.update(conv_taps=0, conv_stream=0, conv_big=0, conv_small=100000000 if prec == "bf16-gemm64" else 0)
        prec = "bf16"
    n, h, w, cin, cout, k, s, p, act, res_mode = case
    ctx = face_ctx_factory(prec, 8, options=tuple(sorted(options.items())))
    rng = np.random.default_rng(cin * 7 + cout)
    x = rng.standard_normal((n, h, w, cin)).astype(F32)
    wt = (rng.standard_normal((cout, cin, k, k)) * np.sqrt(2.0 / (cin * k * k))).astype(F32)
    scale = rng.uniform(0.5, 1.5, cout).astype(F32)
    shift = rng.standard_normal(cout).astype(F32) * F32(0.1)
    oh, ow = (h + 2 * p - k) // s + 1, (w + 2 * p - k) // s + 1
    res = rng.standard_normal((n, oh, ow, cout)).astype(F32) if res_mode else None
    if prec in ("bf16", "fp16"):   # the kernel sees 16-bit operands: compare against the same rounded inputs
        dt = torch.bfloat16 if prec == "bf16" else torch.float16
        bf = lambda a: torch.from_numpy(a).to(dt).float().numpy()
        x, wt = bf(x), bf(wt)
        res = bf(res) if res is not None else None
    got = ctx.conv2d(x, wt, s, p, scale, shift, act, 0.1, res, res_mode)
    y = torch.nn.functional.conv2d(torch.from_numpy(x).permute(0, 3, 1, 2), torch.from_numpy(wt), stride=s,
                                   padding=p).permute(0, 2, 3, 1).double().numpy()
    y = y * scale + shift
    if res_mode == 1:
        y = y + res
    y = {0: lambda v: v, 1: lambda v: np.maximum(v, 0), 2: lambda v: np.where(v > 0, v, 0.1 * v),
         3: lambda v: v / (1 + np.exp(-v))}[act](y)
    if res_mode == 2:
        y = y + res
    tol = {"fp32": 2e-5, "fp16": 1e-3}.get(prec, 2e-2)
    err = np.abs(got - y).max() / (np.abs(y).max() + 1e-6)
    assert got.shape == y.shape
    assert err < tol, f"rel err {err}"


@pytest.mark.parametrize("case", [(2, 20, 24, 256, 256, 3, 1, 1, 0, 0), (1, 40, 40, 512, 128, 1, 1, 0, 0, 0),
                                  (3, 17, 23, 3, 64, 7, 2, 3, 0, 0)])
def test_conv_fp32_split_error_matches_exact_f32(gpu, face_ctx_factory, case):
    """Both split paths' errors against a float64 convolution are at the level of the
    exact-f32 MFMA path's (~1.6e-6 of max|y| at K = 2304): the 3-term bf16 split and the
    scaled fp16 pair are fp32 arithmetic, not a reduced precision (conv_x6.hip)."""
    n, h, w, cin, cout, k, s, p, _, _ = case
    rng = np.random.default_rng(cin + cout + k)
    x = np.maximum(rng.standard_normal((n, h, w, cin)), 0).astype(F32) * F32(3.0)
    wt = (rng.standard_normal((cout, cin, k, k)) * np.sqrt(2.0 / (cin * k * k))).astype(F32)
    y = torch.nn.functional.conv2d(torch.from_numpy(x).permute(0, 3, 1, 2).double(), torch.from_numpy(wt).double(),
                                   stride=s, padding=p).permute(0, 2, 3, 1).numpy()
    errs = {}
    for opts in ((("f32_split", 1),), (("f32_split", 0),), (("f32_split", 2),)):
        ctx = face_ctx_factory("fp32", 8, options=opts)
        got = ctx.conv2d(x, wt, s, p)
        errs[opts] = np.abs(got - y).max() / np.abs(y).max()
    split, exact, pair = errs[(("f32_split", 1),)], errs[(("f32_split", 0),)], errs[(("f32_split", 2),)]
    assert split < 4e-6 and split < 2 * exact + 1e-7, (split, exact)
    assert pair < 4e-6 and pair < 2 * exact + 1e-7, (pair, exact)


BIG_CASES = [
    # 256 x 256-tile phased kernel (conv_big.hip): Cout % 256 == 0, Cin % 64 == 0
    (2, 20, 24, 128, 256, 3, 1, 1, 1, 1),     # 3x3 + residual before ReLU, M tail (960 rows)
    (1, 26, 30, 64, 256, 3, 2, 1, 1, 0),      # stride 2, two K tiles per tap row
    (1, 33, 31, 256, 512, 1, 1, 0, 0, 2),     # 1x1, two N tiles, residual after activation
    (2, 9, 11, 512, 256, 3, 1, 1, 2, 0),      # K = 4608 (72 K tiles), leaky
]


@pytest.mark.parametrize("case", BIG_CASES)
def test_conv_big_matches_torch(gpu, face_ctx_factory, case):
    """Force the phased 256x256 kernel onto small shapes (option conv_big = min tiles)."""
    test_conv_matches_torch(gpu, face_ctx_factory, "bf16", case,
                            options=dict(conv_big=1, conv_big_kmin=0, conv_stream=0))


# ------------------------------------------------------------------ fused bottleneck
BLOCK_CASES = [
    # (n, h, w, cin, downsample)
    (2, 16, 32, 256, False),     # whole 8x16 tiles
    (1, 21, 37, 256, False),     # ragged tiles on both axes
    (2, 13, 18, 64, True),       # layer1.0: cin 64 + downsample branch
    (8, 96, 160, 256, False),    # 960 tiles: several per persistent workgroup (block32_pipe's buffers cycle)
    (1, 8, 5, 64, True),         # narrower than one tile
    (1, 40, 40, 256, False),     # 3x3 halo across interior tile seams
]


def _bn(rng, c):
    return np.concatenate([rng.uniform(0.5, 1.5, c), rng.standard_normal(c) * 0.1]).astype(F32)


@pytest.mark.parametrize("case", BLOCK_CASES)
def test_bottleneck_fused_matches_torch_and_chain(gpu, face_ctx_factory, case):
    """block.hip (one kernel per bottleneck) against (a) a torch fp32 bottleneck on the
    same bf16-rounded operands with t1/t2 rounded to bf16 as the kernels store them
    (2e-2 relative, the bf16 bar), and (b) the conv-by-conv chain of the same library
    (same bf16 weights, only the f32 summation order differs: 1e-2 relative)."""
    n, h, w, cin, ds = case
    ctx = face_ctx_factory("bf16", 8)
    rng = np.random.default_rng(h * 100 + w + cin)
    bf = lambda a: torch.from_numpy(np.ascontiguousarray(a, F32)).bfloat16().float().numpy()
    he = lambda co, ci, k: (rng.standard_normal((co, ci, k, k)) * np.sqrt(2.0 / (ci * k * k))).astype(F32)
    x = bf(rng.standard_normal((n, h, w, cin)).astype(F32))
    w1, w2, w3 = bf(he(64, cin, 1)), bf(he(64, 64, 3)), bf(he(256, 64, 1))
    b1, b2, b3 = _bn(rng, 64), _bn(rng, 64), _bn(rng, 256)
    wd, bd = (bf(he(256, cin, 1)), _bn(rng, 256)) if ds else (None, None)
    got = ctx.bottleneck(x, w1, b1, w2, b2, w3, b3, wd, bd, fused=True)
    chain = ctx.bottleneck(x, w1, b1, w2, b2, w3, b3, wd, bd, fused=False)

    T = lambda a: torch.from_numpy(a)
    conv = lambda v, wt, p: torch.nn.functional.conv2d(v, T(wt), padding=p)
    aff = lambda v, b, c: v * T(b[:c]).view(1, c, 1, 1) + T(b[c:]).view(1, c, 1, 1)
    rb = lambda v: v.bfloat16().float()
    xt = T(x).permute(0, 3, 1, 2)
    t1 = rb(torch.relu(aff(conv(xt, w1, 0), b1, 64)))
    t2 = rb(torch.relu(aff(conv(t1, w2, 1), b2, 64)))
    idt = aff(conv(xt, wd, 0), bd, 256) if ds else xt
    ref = torch.relu(aff(conv(t2, w3, 0), b3, 256) + idt).permute(0, 2, 3, 1).numpy()
    scale = np.abs(ref).max() + 1e-6
    assert got.shape == ref.shape
    assert np.abs(got - ref).max() / scale < 2e-2
    assert np.abs(got - chain).max() / scale < 1e-2
    assert np.mean(got == chain) > 0.95        # mostly bit-identical after bf16 rounding


@pytest.mark.parametrize("case", BLOCK_CASES)
def test_bottleneck_fp32_fused_matches_float64(gpu, face_ctx_factory, case):
    """block32.hip (the fp32 plan's one-kernel layer1 bottleneck: fp16 pairs, t1 / t2
    scaled per tile in LDS) against a float64 torch bottleneck on the same f32 inputs,
    beside the conv-by-conv fp32 chain of the same library (per-frame scales): both sit
    at f32 rounding (< 2e-6 of the output range), the fused error within 2x the chain's."""
    n, h, w, cin, ds = case
    ctx = face_ctx_factory("fp32", 8)
    rng = np.random.default_rng(h * 100 + w + cin + 7)
    he = lambda co, ci, k: (rng.standard_normal((co, ci, k, k)) * np.sqrt(2.0 / (ci * k * k))).astype(F32)
    x = np.maximum(rng.standard_normal((n, h, w, cin)), 0).astype(F32)      # a ReLU output, as in the net
    w1, w2, w3 = he(64, cin, 1), he(64, 64, 3), he(256, 64, 1)
    b1, b2, b3 = _bn(rng, 64), _bn(rng, 64), _bn(rng, 256)
    wd, bd = (he(256, cin, 1), _bn(rng, 256)) if ds else (None, None)
    got = ctx.bottleneck(x, w1, b1, w2, b2, w3, b3, wd, bd, fused=True)
    chain = ctx.bottleneck(x, w1, b1, w2, b2, w3, b3, wd, bd, fused=False)

    T = lambda a: torch.from_numpy(np.asarray(a, np.float64))
    conv = lambda v, wt, p: torch.nn.functional.conv2d(v, T(wt), padding=p)
    aff = lambda v, b, c: v * T(b[:c]).view(1, c, 1, 1) + T(b[c:]).view(1, c, 1, 1)
    xt = T(x).permute(0, 3, 1, 2)
    t1 = torch.relu(aff(conv(xt, w1, 0), b1, 64))
    t2 = torch.relu(aff(conv(t1, w2, 1), b2, 64))
    idt = aff(conv(xt, wd, 0), bd, 256) if ds else xt
    ref = torch.relu(aff(conv(t2, w3, 0), b3, 256) + idt).permute(0, 2, 3, 1).numpy()
    scale = np.abs(ref).max()
    e_fused = np.abs(got - ref).max() / scale
    e_chain = np.abs(chain - ref).max() / scale
    print(f"fp32 bottleneck {case}: fused {e_fused:.2e}, chain {e_chain:.2e}")
    assert got.shape == ref.shape
    assert e_fused < 2e-6 and e_chain < 2e-6
    assert e_fused <= 2 * e_chain + 1e-7


# ------------------------------------------------------------------ post-processing
def _heads(rng, n, A, bias):
    loc = (rng.standard_normal((n, A, 4)) * 1.5).astype(F32)
    conf = rng.standard_normal((n, A, 2)).astype(F32)
    conf[..., 1] += F32(bias)
    return loc, conf


def _oracle_post(loc, conf, img_h, img_w, thr=0.5, iou=0.4):
    pri = oanchors.get_anchors((640, 640))
    res = []
    for b in range(loc.shape[0]):
        idx, boxes, sc = obbox.postprocess_frame(loc[b], conf[b], pri, thr, iou)
        fb = obbox.correct_and_scale(boxes, img_h, img_w)
        res.append((idx, fb, obbox.truncate_boxes(fb), sc))
    return res


@pytest.mark.parametrize("bias,hw", [(-4.0, (1080, 1920)), (-2.0, (720, 1280)), (-1.0, (640, 640)),
                                     (0.3, (2160, 3840)), (-9.0, (1080, 1920))])
def test_postprocess_bit_exact(gpu, face_ctx_factory, bias, hw):
    """Same loc/conf into both sides -> identical keep lists, float boxes, int boxes, scores.
    bias -4 ~ 2 % candidates (LDS path); -1 / 0.3 put > 2048 candidates through the global path."""
    ctx = face_ctx_factory("fp32", 8)
    rng = np.random.default_rng(int(abs(bias) * 100))
    loc, conf = _heads(rng, 3, 16800, bias)
    got = ctx.postprocess(loc, conf, hw, cap=16800)
    exp = _oracle_post(loc, conf, *hw)
    for b in range(3):
        xi, xf, sc, lab = got.frame(b)
        e_idx, e_f, e_i, e_sc = exp[b]
        assert int(got.count[b]) == len(e_idx)
        np.testing.assert_array_equal(lab, e_idx)
        np.testing.assert_array_equal(xf, e_f)
        np.testing.assert_array_equal(xi, e_i)
        np.testing.assert_array_equal(sc, e_sc)


def test_postprocess_ties_and_capacity(gpu, face_ctx_factory):
    from vdmi import _lib
    ctx = face_ctx_factory("fp32", 8)
    A = 16800
    loc = np.zeros((1, A, 4), F32)
    conf = np.zeros((1, A, 2), F32)
    conf[0, :, 0] = 1.0             # background everywhere except the strided anchors
    conf[0, ::7, 1] = 2.0           # many exactly-equal scores: stable order decides
    conf[0, ::11, 1] = 3.0
    got = ctx.postprocess(loc, conf, (1080, 1920), cap=8192)
    e = _oracle_post(loc, conf, 1080, 1920)[0]
    np.testing.assert_array_equal(got.frame(0)[3], e[0])
    # a cap below the keep count is not an error: count is complete, the arrays hold
    # the first cap boxes, and vd_read_boxes returns the complete list
    small = ctx.postprocess(loc, conf, (1080, 1920), cap=4)
    assert int(small.count[0]) == len(e[0]) > 4
    np.testing.assert_array_equal(small.frame(0)[3], e[0][:4])
    full = ctx.read_boxes(_lib.VD_NET_RETINAFACE, 1)
    assert full.cap == len(e[0])
    np.testing.assert_array_equal(full.frame(0)[3], e[0])
    np.testing.assert_array_equal(full.frame(0)[0], e[2])


S2_CASES = [
    # fp32 stride-2 3x3 convs on the phase halos (option x6_halo_s2): odd input dims (the odd
    # row / column past the input), several frames per tile, N = 64 / 128 / 256-wide tiles,
    # residual, the widest phase halo (Wo = 254)
    (3, 17, 15, 32, 64, 3, 2, 1, 1, 0),
    (2, 16, 16, 64, 128, 3, 2, 1, 1, 1),
    (1, 5, 507, 32, 128, 3, 2, 1, 2, 0),
    (1, 9, 8, 256, 512, 3, 2, 1, 1, 0),
    (4, 224, 224, 32, 256, 3, 2, 1, 1, 0),    # >= 192 256-wide tiles: the 256 x 256 halo tile
]


@pytest.mark.parametrize("case", S2_CASES)
def test_conv_halo_s2_matches_torch_and_batch_invariant(gpu, face_ctx_factory, case):
    """Phase-halo stride-2 convs (conv_x6_halo_kernel<..., S2>) within the fp32 tolerance of
    torch, like the tap-major tiles they replace (x6_halo_s2 = 0); every output's K order
    is fixed, so a frame's outputs do not depend on the batch around it (bit-identical
    to the frame run alone)."""
    for s2 in (1, 0):
        test_conv_matches_torch(gpu, face_ctx_factory, "fp32", case, options=dict(x6_halo_s2=s2))
    n, h, w, cin, cout, k, s, p, act, res_mode = case
    if n == 1:
        return
    ctx = face_ctx_factory("fp32", 8, options=(("x6_halo_s2", 1),))
    rng = np.random.default_rng(cin + cout)
    x = np.maximum(rng.standard_normal((n, h, w, cin)), 0).astype(F32)
    wt = (rng.standard_normal((cout, cin, k, k)) * np.sqrt(2.0 / (9 * cin))).astype(F32)
    scale = rng.uniform(0.5, 1.5, cout).astype(F32)
    shift = rng.standard_normal(cout).astype(F32) * F32(0.1)
    oh, ow = (h - 1) // 2 + 1, (w - 1) // 2 + 1
    res = rng.standard_normal((n, oh, ow, cout)).astype(F32) if res_mode else None
    full = ctx.conv2d(x, wt, s, p, scale, shift, act, 0.1, res, res_mode)
    for b in range(n):
        one = ctx.conv2d(x[b:b + 1], wt, s, p, scale, shift, act, 0.1,
                         None if res is None else res[b:b + 1], res_mode)
        assert np.array_equal(one[0], full[b]), b


TR_CASES = [
    # 1x1 convs on the TR tiles (option x6_gemm1x1): 256 x 256 (Cout % 256, >= 192 tiles), 256 x 128,
    # 128 x 128 (Cout 128, K <= 512); M tails, stride 2, residual before / after the activation
    (2, 37, 41, 512, 256, 1, 1, 0, 1, 1),
    (1, 33, 35, 1024, 512, 1, 2, 0, 0, 0),
    (3, 19, 23, 512, 128, 1, 1, 0, 1, 0),
    (1, 21, 19, 256, 384, 1, 1, 0, 2, 2),
    (2, 45, 47, 512, 2048, 1, 1, 0, 1, 1),
]


@pytest.mark.parametrize("case", TR_CASES)
def test_conv_tr_tiles_bit_identical(gpu, face_ctx_factory, case):
    """The TR tiles (D^T accumulators, register epilogue) compute the same products in
    the same order as the untransposed tiles: outputs (and the per-frame max slots the
    hook checks) are bit-identical, and within the fp32 tolerance of torch."""
    n, h, w, cin, cout, k, s, p, act, res_mode = case
    rng = np.random.default_rng(cin + 3 * cout)
    x = np.maximum(rng.standard_normal((n, h, w, cin)), 0).astype(F32)
    wt = (rng.standard_normal((cout, cin, k, k)) * np.sqrt(2.0 / cin)).astype(F32)
    scale = rng.uniform(0.5, 1.5, cout).astype(F32)
    shift = rng.standard_normal(cout).astype(F32) * F32(0.1)
    oh, ow = (h - 1) // s + 1, (w - 1) // s + 1
    res = rng.standard_normal((n, oh, ow, cout)).astype(F32) if res_mode else None
    outs = []
    for tr in (0, 1):
        ctx = face_ctx_factory("fp32", 8, options=(("x6_gemm1x1", tr), ("x6_stream", 0)))
        outs.append(ctx.conv2d(x, wt, s, p, scale, shift, act, 0.1, res, res_mode))
    assert np.array_equal(outs[0], outs[1])
    test_conv_matches_torch(gpu, face_ctx_factory, "fp32", case, options=dict(x6_gemm1x1=1, x6_stream=0))


@pytest.mark.parametrize("mapon", [0, 1])
def test_mosaic_output_forms_match_oracle(gpu, mapon):
    """Option mosaic_map: 1 (default) = the band output pass with per-band vector maps;
    0 = the generic per-pixel path. Both exact against the oracle on overlapping /
    nested boxes, > 256 boxes (no cell table), a cell-table overflow and frames with
    no boxes."""
    import vdmi
    from vdmi import mosaic_frames, synth
    ctx = vdmi.Context(precision="bf16", max_batch=4, options={"mosaic_map": mapon})
    try:
        rng = np.random.default_rng(21)
        frames = synth.frames(4, 480, 720, seed=21)
        nested = [(10 + 3 * i, 5 + 9 * i, 700 - 2 * i, 470 - i) for i in range(25)]
        many = [tuple(int(v) for v in (x, y, x + rng.integers(4, 60), y + rng.integers(4, 60)))
                for x, y in zip(rng.integers(-20, 720, 300), rng.integers(-20, 480, 300))]
        boxes = [_rand_boxes(rng, 1, 480, 720, 30)[0], nested, many, []]
        for level in (1, 3, 8):
            got = mosaic_frames(frames, boxes, level, ctx=ctx)
            for i in range(4):
                np.testing.assert_array_equal(got[i], omosaic.mosaic_frame(frames[i], boxes[i], level))
    finally:
        ctx.close()


@pytest.mark.parametrize("fused,rows,gather", [(0, 0, 0), (1, 0, 0), (1, 4, 0), (1, 8, 0), (1, 16, 0), (1, 24, 0),
                                               (1, 32, 0), (1, 0, 1), (1, 8, 1)])
def test_mosaic_fused_and_two_launch_paths_match_oracle(gpu, fused, rows, gather):
    """Option mosaic_fused: 1 (default) = one launch, the output pass walks and gathers
    its bands' cells itself; 0 = cell-table kernel + output pass; the fused pass at
    4 / 8 / 16 / 24 / 32 rows per band (option mosaic_rows), with the band cells'
    source loads batched (option mosaic_gather). All exact on random
    boxes (incl. degenerate / off-frame ones), nested chains, a level-2 band whose cells
    exceed the LDS slice, > MAPBOX boxes in a band and > BOX_FAST boxes in a frame."""
    import vdmi
    from vdmi import mosaic_frames, synth
    ctx = vdmi.Context(precision="bf16", max_batch=4,
                       options={"mosaic_fused": fused, "mosaic_rows": rows, "mosaic_gather": gather})
    try:
        rng = np.random.default_rng(17 + fused)
        frames = synth.frames(3, 1080, 1920, seed=21)
        cases = [(_rand_boxes(rng, 3, 1080, 1920, 40), 8)]
        cases.append(([[(10 + 3 * i, 5 + 9 * i, 1900 - 2 * i, 1070 - i) for i in range(25)],
                       [(100, 200, 1100, 600), (900, 500, 1500, 900)],
                       [(40 * i, 300 + i, 40 * i + 60, 360 + 2 * i) for i in range(45)]], 2))
        many = [tuple(int(v) for v in (x, y, x + rng.integers(4, 90), y + rng.integers(4, 90)))
                for x, y in zip(rng.integers(-20, 1920, 300), rng.integers(-20, 1080, 300))]
        cases.append(([many, many[:200], []], 8))
        for boxes, level in cases:
            got = mosaic_frames(frames, boxes, level, ctx=ctx)
            for i in range(3):
                np.testing.assert_array_equal(got[i], omosaic.mosaic_frame(frames[i], boxes[i], level),
                                              err_msg=f"frame {i} level {level}")
    finally:
        ctx.close()
