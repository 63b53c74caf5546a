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
