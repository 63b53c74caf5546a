"""JPEG frame encode (the cv2.imwrite of every processed frame,
combine_detect.py:174-180, whose output create_video reads back).

CPU: the oracle (oracle/jpeg_enc.py, libjpeg-turbo's compressor restated) is pinned
byte for byte against Pillow's libjpeg-turbo encoder at several qualities, all three
samplings and ragged sizes (partial MCUs: dummy blocks, edge replication, the
downsampling bias), and its output decodes through the decode oracle to Pillow's
decode of Pillow's bytes. The library exports vd_jpeg_encode (GPU test: test_gpu_jpeg).
Parity with cv2's header bytes is unpinned (cv2 is absent; both are libjpeg-turbo).
"""
import io

import numpy as np
import pytest
from PIL import Image

from oracle import jpeg as ojpeg
from oracle import jpeg_enc

ENC_CASES = [   # (h, w, quality, subsampling: 0 = 4:4:4, 1 = 4:2:2, 2 = 4:2:0)
    (16, 16, 95, 2), (17, 23, 95, 2), (8, 8, 75, 0), (33, 47, 90, 1), (40, 56, 95, 2), (31, 45, 85, 2),
    (64, 96, 50, 0), (9, 31, 100, 2), (25, 7, 30, 1), (48, 64, 95, 1),
]


def frame(h, w, seed=0):
    """Block noise + gradients + a flat patch (long zero runs, ZRL codes)."""
    rng = np.random.default_rng(seed + h * 131 + w)
    base = rng.integers(0, 256, ((h + 3) // 4, (w + 3) // 4, 3))
    img = np.repeat(np.repeat(base, 4, 0), 4, 1)[:h, :w].astype(np.float64)
    img = img * 0.6 + np.arange(w)[None, :, None] * 0.5 + np.arange(h)[:, None, None] * 0.3
    img[: h // 3, : w // 3] = 77
    return img.clip(0, 255).astype(np.uint8)


def pillow_jpeg(img, q, sub):
    b = io.BytesIO()
    Image.fromarray(img).save(b, "JPEG", quality=q, subsampling=sub)
    return b.getvalue()


@pytest.mark.parametrize("case", ENC_CASES)
def test_encode_oracle_matches_pillow_bytes(case):
    h, w, q, sub = case
    img = frame(h, w)
    assert jpeg_enc.encode(img, q, sub) == pillow_jpeg(img, q, sub)


def test_encode_oracle_noise_and_flat():
    rng = np.random.default_rng(7)
    noise = rng.integers(0, 256, (24, 40, 3), dtype=np.uint8)         # every coefficient nonzero
    flat = np.full((24, 40, 3), 200, np.uint8)                         # DC only, EOB everywhere
    for img in (noise, flat):
        assert jpeg_enc.encode(img, 95, 2) == pillow_jpeg(img, 95, 2)


def test_encode_roundtrip_through_decode_oracle():
    img = frame(40, 56, seed=3)
    d = jpeg_enc.encode(img, 95, 2)
    got = ojpeg.decode(d)
    exp = np.asarray(Image.open(io.BytesIO(d)).convert("RGB"))
    np.testing.assert_array_equal(got, exp)
    assert np.abs(got.astype(int) - img).mean() < 16                 # 4:2:0 colour edges of block noise


def test_quant_tables_and_reciprocals():
    q = jpeg_enc.quant_table(jpeg_enc.STD_LUMA, 95)
    assert q[0] == 2 and q[1] == 1 and q.max() <= 255                 # (16 * 10 + 50) // 100 = 2
    for d in (8, 16, 24, 88, 792, 2040):                              # power-of-two and general divisors
        fq, c, r = jpeg_enc.reciprocal(d)
        for x in range(0, 20000, 7):
            assert ((x + c) * fq) >> r == (x + d // 2) // d           # == rounded division here


def test_library_exports_encode():
    from vdmi import _lib
    lib = _lib.load()
    assert hasattr(lib, "vd_jpeg_encode")
