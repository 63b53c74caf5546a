"""vd_jpeg_decode / vd_jpeg_encode on the GPU: bit-exact against Pillow's libjpeg-turbo (and the
oracle) for every supported layout, batched 1080p frames decoded straight into
device memory, and those frames through vd_process identical to host-decoded ones."""
import io

import numpy as np
import pytest
from PIL import Image

from test_jpeg import CASES, make_jpeg, pillow_rgb

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def jctx(gpu):
    import vdmi
    from vdmi import weights
    ctx = vdmi.Context(precision="fp32", max_batch=8)
    ctx.load_weights(0, weights.retinaface_state_dict(0))
    yield ctx
    ctx.close()


@pytest.mark.parametrize("case", CASES + [(40, 56, 90, 2, 0, 3)])
def test_decode_matches_pillow(jctx, case):
    h, w, q, sub = case[:4]
    d = make_jpeg(h, w, q, sub, restart=case[5] if len(case) > 5 else None)
    got = jctx.jpeg_decode([d, d])
    exp = pillow_rgb(d)
    np.testing.assert_array_equal(got[0], exp)
    np.testing.assert_array_equal(got[1], exp)


@pytest.fixture(scope="module")
def jctx_host_dec(gpu):
    """Entropy decode on host threads (option jdec_gpu=0): the pre-device path, pinned
    to Pillow by the tests above in earlier rounds."""
    import vdmi
    ctx = vdmi.Context(precision="fp32", max_batch=8, options={"jdec_gpu": 0})
    yield ctx
    ctx.close()


@pytest.mark.parametrize("sync", [128, 0, 2])
@pytest.mark.parametrize("chunk", [16, 48, 256])
@pytest.mark.parametrize("case", CASES)
def test_device_entropy_small_chunks_matches_pillow(gpu, case, chunk, sync):
    """jpeg_dec.hip with tiny chunks (option jdec_chunk): every frame is cut into many
    speculatively decoded chunks, so block boundaries, the block-in-MCU phase and DC
    predictors must all be recovered by the resynchronisation passes -- with the early
    stop at the previous trajectory (jdec_sync states recorded per chunk; 2: lists
    shorter than most chunks) or without it (0); the result is still libjpeg-turbo's
    decode bit for bit."""
    import vdmi
    h, w, q, sub = case[:4]
    ctx = vdmi.Context(precision="fp32", max_batch=4, options={"jdec_chunk": chunk, "jdec_sync": sync})
    try:
        ds = [make_jpeg(h, w, q, sub, seed=s) for s in range(3)]
        got = ctx.jpeg_decode(ds)
        for g, d in zip(got, ds):
            np.testing.assert_array_equal(g, pillow_rgb(d))
    finally:
        ctx.close()


@pytest.mark.parametrize("noise", [False, True])
def test_device_entropy_1080p_equals_host_threads(jctx, jctx_host_dec, noise):
    """1080p q95 4:2:0 frames (ffmpeg-split shape), structured and noise (2.4 MB of
    entropy data per frame, ~1200 chunks): device and host entropy stages give the
    same frames, equal to Pillow's decode."""
    from vdmi import synth
    fr = synth.frames(3, 1080, 1920, seed=21)
    if not noise:
        fr = np.repeat(np.repeat(fr[:, ::4, ::4], 4, 1), 4, 2)
    jp = []
    for f in fr:
        b = io.BytesIO()
        Image.fromarray(f).save(b, "JPEG", quality=95)
        jp.append(b.getvalue())
    dev = jctx.jpeg_decode(jp)
    assert jctx.jdec_passes() >= 2, "the device entropy stage ran"
    host = jctx_host_dec.jpeg_decode(jp)
    np.testing.assert_array_equal(dev, host)
    np.testing.assert_array_equal(dev[0], pillow_rgb(jp[0]))


def test_device_entropy_damaged_stream_same_as_host(jctx, jctx_host_dec):
    """Damaged entropy data (bytes overwritten mid-scan, a truncated scan): the device
    stage flags the stream and the host stage decides, so the result (or the error) is
    the host decoder's."""
    import vdmi
    d = bytearray(make_jpeg(64, 96, 95, 2, seed=3))
    sos = d.index(b"\xff\xda")
    for k in range(sos + 40, sos + 60):
        d[k] = (d[k] * 37 + 11) & 0xFF
        if d[k] == 0xFF:
            d[k] = 0xFE
    cut = bytes(d[:sos + 100])
    for blob in (bytes(d), cut):
        try:
            h = jctx_host_dec.jpeg_decode([blob])
        except vdmi.VdError as e:
            with pytest.raises(vdmi.VdError):
                jctx.jpeg_decode([blob])
            continue
        np.testing.assert_array_equal(jctx.jpeg_decode([blob]), h)


def _video_frames(n, h=1080, w=1920, q=95):
    """ffmpeg-like frames: synthetic 1080p RGB encoded by libjpeg (Pillow) at q95, 4:2:0."""
    from vdmi import synth
    fr = synth.frames(n, h, w, seed=5)
    out = []
    for f in fr:
        b = io.BytesIO()
        Image.fromarray(f).save(b, "JPEG", quality=q)
        out.append(b.getvalue())
    return out


def test_batch_1080p_device_decode_and_process(jctx):
    import torch
    from vdmi import _lib
    jp = _video_frames(6)
    dev = torch.device("cuda:0")
    d = torch.empty((6, 1080, 1920, 3), dtype=torch.uint8, device=dev)
    jctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    try:
        jctx.jpeg_decode(jp, out=d)
        torch.cuda.synchronize()
        host = np.stack([pillow_rgb(j) for j in jp])
        np.testing.assert_array_equal(d.cpu().numpy(), host)
        # decoded-on-device frames through the hot path == host-decoded frames
        out_d, faces_d, _ = jctx.process(d)
        torch.cuda.synchronize()
        lists_d = jctx.read_boxes(_lib.VD_NET_RETINAFACE, 6)
        out_h, faces_h, _ = jctx.process(host)
        lists_h = jctx.read_boxes(_lib.VD_NET_RETINAFACE, 6)
        np.testing.assert_array_equal(out_d.cpu().numpy(), out_h)
        np.testing.assert_array_equal(lists_d.count, lists_h.count)
        for b in range(6):
            np.testing.assert_array_equal(lists_d.frame(b)[0], lists_h.frame(b)[0])
    finally:
        jctx.set_stream(None)


# ------------------------------------------------------------------ encode (vd_jpeg_encode)
from test_jpeg_enc import ENC_CASES, frame as enc_frame, pillow_jpeg  # noqa: E402


@pytest.mark.parametrize("case", ENC_CASES)
def test_encode_matches_pillow_bytes(jctx, case):
    h, w, q, sub = case
    imgs = np.stack([enc_frame(h, w, seed=s) for s in range(3)])
    got = jctx.jpeg_encode(imgs, quality=q, subsampling=sub)
    for img, g in zip(imgs, got):
        assert g == pillow_jpeg(img, q, sub)


def test_encode_noise_needs_the_retry_capacity(jctx):
    rng = np.random.default_rng(11)
    noise = rng.integers(0, 256, (2, 48, 64, 3), dtype=np.uint8)
    got = jctx.jpeg_encode(noise, quality=100, subsampling=0)       # > 3 B/pixel: second capacity pass
    for img, g in zip(noise, got):
        assert g == pillow_jpeg(img, 100, 0)


def test_encode_1080p_from_device_frames_after_process(jctx):
    """The reference's per-frame write (cv2.imwrite, q95, 4:2:0) of mosaicked frames
    that never leave the GPU: vd_process output -> vd_jpeg_encode from device memory;
    bytes equal Pillow's encode of the same frames, and decode back bit-exactly."""
    import torch
    from vdmi import synth
    dev = torch.device("cuda:0")
    fr = torch.from_numpy(synth.frames(4, 1080, 1920, seed=9)).to(dev)
    out, _, _ = jctx.process(fr)
    torch.cuda.synchronize()
    got = jctx.jpeg_encode(out, quality=95, subsampling=2)
    host = out.cpu().numpy()
    for img, g in zip(host, got):
        assert g == pillow_jpeg(img, 95, 2)
    back = jctx.jpeg_decode(got)
    np.testing.assert_array_equal(back, np.stack([pillow_rgb(g) for g in got]))


@pytest.fixture(scope="module")
def hctx(gpu):
    import vdmi
    ctx = vdmi.Context(precision="fp32", max_batch=8, options={"jenc_gpu": 0})
    yield ctx
    ctx.close()


@pytest.mark.parametrize("case", ENC_CASES + [(1080, 1920, 95, 2), (1080, 1920, 100, 0), (37, 1001, 75, 1)])
@pytest.mark.parametrize("noise", [False, True])
def test_encode_device_entropy_equals_host_threads(jctx, hctx, case, noise):
    """Huffman coding on the device (default, option jenc_gpu; jpeg_enc.hip: per-unit
    code lengths, a per-frame scan, atomic-OR word writes at neighbour boundaries, a
    stuffing pass) writes the same bytes as the host threads' sequential coder
    (jpeg_enc.cpp, pinned to Pillow) -- dummy blocks, long zero runs (ZRL), 0xFF
    stuffing and noise frames of several MB included."""
    h, w, q, sub = case
    if noise:
        rng = np.random.default_rng(h * w + q)
        imgs = rng.integers(0, 256, (2, h, w, 3), dtype=np.uint8)
    else:
        imgs = np.stack([enc_frame(h, w, seed=s) for s in range(2)])
    dev = jctx.jpeg_encode(imgs, quality=q, subsampling=sub)
    host = hctx.jpeg_encode(imgs, quality=q, subsampling=sub)
    assert [len(d) for d in dev] == [len(x) for x in host]
    for d, x in zip(dev, host):
        assert d == x
    if h * w <= 64 * 64:
        for img, d in zip(imgs, dev):
            assert d == pillow_jpeg(img, q, sub)
