"""JPEG frame decode (the cv2.imread of the ffmpeg-split
frames, combine_detect.py:167-172).

CPU: the oracle (oracle/jpeg.py, libjpeg-turbo's default decode restated) is
pinned bit-exactly against Pillow's libjpeg-turbo on frames of every supported
layout (4:2:0 / 4:2:2 / 4:4:4 / grayscale, odd sizes, several qualities, restart
markers); the library's host-only parser reports the geometry.
GPU: vd_jpeg_decode is bit-exact against both, and frames decoded on the device
feed vd_process with the same boxes and pixels as host-decoded frames.
Parity with cv2 itself is unpinned (cv2 is absent; it uses libjpeg-turbo too).
"""
import io

import numpy as np
import pytest
from PIL import Image

from oracle import jpeg as ojpeg

CASES = [   # (h, w, quality, subsampling: 0 = 4:4:4, 1 = 4:2:2, 2 = 4:2:0, "L" = grayscale)
    (48, 64, 95, 2), (50, 70, 75, 2), (37, 53, 90, 1), (40, 40, 85, 0), (33, 47, 95, 2), (64, 96, 50, 2),
    (31, 45, 92, "L"), (72, 88, 100, 2),
]


def make_jpeg(h, w, q, sub, seed=0, restart=None):
    """Structured synthetic content (block noise + gradients) through Pillow's encoder."""
    from vdmi import synth
    base = synth.frames(1, (h + 3) // 4, (w + 3) // 4, seed=seed + h * w)[0]
    img = np.repeat(np.repeat(base, 4, 0), 4, 1)[:h, :w].astype(np.float32)
    img = (img * 0.6 + np.arange(w)[None, :, None] * 0.3 + np.arange(h)[:, None, None] * 0.2).clip(0, 255)
    img = img.astype(np.uint8)
    b = io.BytesIO()
    kw = dict(quality=q)
    if restart:
        kw["restart_marker_blocks"] = restart
    if sub == "L":
        Image.fromarray(img[..., 0]).save(b, "JPEG", **kw)
    else:
        Image.fromarray(img).save(b, "JPEG", subsampling=sub, **kw)
    return b.getvalue()


def pillow_rgb(data):
    return np.asarray(Image.open(io.BytesIO(data)).convert("RGB"))


@pytest.mark.parametrize("case", CASES)
def test_oracle_matches_pillow(case):
    d = make_jpeg(*case)
    np.testing.assert_array_equal(ojpeg.decode(d), pillow_rgb(d))


def test_oracle_restart_markers():
    d = make_jpeg(40, 56, 90, 2, restart=3)
    assert b"\xff\xdd" in d                       # a DRI segment was written
    np.testing.assert_array_equal(ojpeg.decode(d), pillow_rgb(d))


def test_library_jpeg_info_and_errors():
    import vdmi
    d = make_jpeg(37, 53, 90, 1)
    assert vdmi.jpeg_info(d) == (37, 53, 3)
    assert vdmi.jpeg_info(make_jpeg(31, 45, 92, "L")) == (31, 45, 1)
    with pytest.raises(vdmi.VdError):
        vdmi.jpeg_info(b"not a jpeg at all")
    b = io.BytesIO()
    Image.fromarray(np.zeros((16, 16, 3), np.uint8)).save(b, "JPEG", progressive=True)
    with pytest.raises(vdmi.VdError, match="progressive"):
        vdmi.jpeg_info(b.getvalue())


def _lib_coefficients(d):
    import ctypes
    from vdmi import _lib
    lib = _lib.load()
    buf = ctypes.create_string_buffer(d, len(d))
    nb = ctypes.c_int()
    _lib.check(lib.vdt_jpeg_coefficients(buf, len(d), None, 0, ctypes.byref(nb)))
    out = np.zeros((nb.value, 64), np.int16)
    _lib.check(lib.vdt_jpeg_coefficients(buf, len(d), out.ctypes.data, nb.value, ctypes.byref(nb)))
    return out


@pytest.mark.parametrize("case", CASES + [(40, 56, 90, 2, 0, 3), (200, 304, 95, 2, 4)])
def test_library_entropy_decode_matches_oracle(case):
    """The product's host Huffman stage (jpeg_host.cpp, 9-bit lookahead, byte
    unstuffing, restart markers) yields the oracle's coefficients exactly."""
    h, w, q, sub = case[:4]
    d = make_jpeg(h, w, q, sub, seed=case[4] if len(case) > 4 else 0,
                  restart=case[5] if len(case) > 5 else None)
    j = ojpeg.parse(d)
    exp = np.concatenate([c.reshape(-1, 64) for c in ojpeg.coefficients(j)])
    np.testing.assert_array_equal(_lib_coefficients(d).astype(np.int64), exp)


# --------------------------------------------------------------- malformed input
def _segments(d):
    """[(marker, offset of the FF byte, segment length)] up to SOS."""
    out, o = [], 2
    while o + 4 <= len(d):
        m, ln = d[o + 1], (d[o + 2] << 8) | d[o + 3]
        out.append((m, o, ln))
        if m == 0xDA:
            break
        o += 2 + ln
    return out


def _seg(d, marker):
    return next((o, ln) for m, o, ln in _segments(d) if m == marker)


def _oversubscribed_dht(d):
    """Move three codes of some length to length 1: 3 one-bit codes cannot exist."""
    b = bytearray(d)
    o, _ = _seg(d, 0xC4)
    counts = o + 5                       # FF C4 Lh Ll Tc/Th counts[16]
    src = next(l for l in range(1, 16) if b[counts + l] >= 3)
    b[counts + src] -= 3
    b[counts] += 3
    return bytes(b)


def _truncated_sos(d):
    b = bytearray(d)
    o, _ = _seg(d, 0xDA)
    b[o + 2], b[o + 3] = 0, 3            # Ls = 3: room for Ns only
    return bytes(b)


def _duplicate_component(d):
    b = bytearray(d)
    o, _ = _seg(d, 0xC0)
    b[o + 10 + 3] = b[o + 10]            # component 2 id = component 1 id
    return bytes(b)


def _second_sof(d):
    o, ln = _seg(d, 0xC0)
    sof = d[o:o + 2 + ln]
    s, _ = _seg(d, 0xDA)
    return d[:s] + sof + d[s:]


@pytest.mark.parametrize("mutate,msg", [(_oversubscribed_dht, "Huffman"), (_truncated_sos, "SOS"),
                                        (_duplicate_component, "duplicate"), (_second_sof, "more than one")])
def test_library_rejects_malformed_jpeg(mutate, msg):
    """The host parser (jpeg_host.cpp) refuses headers that would otherwise index
    past its tables: an over-subscribed DHT (fills past the 2048-entry lookahead),
    a short SOS, duplicate component ids (unassigned table indices), two SOFs."""
    import vdmi
    d = mutate(make_jpeg(48, 64, 95, 2))
    with pytest.raises(vdmi.VdError, match=msg):
        vdmi.jpeg_info(d)
    with pytest.raises(vdmi.VdError):
        _lib_coefficients(d)


def test_library_rejects_truncated_scan_without_crash():
    """Entropy data cut short: the bit reader feeds zeros past the end (as libjpeg
    does) -- the call returns (an error or zero-padded coefficients), never reads past."""
    import vdmi
    d = make_jpeg(64, 96, 95, 2)
    o, ln = _seg(d, 0xDA)
    cut = d[:o + 2 + ln + 40]
    try:
        _lib_coefficients(cut)
    except vdmi.VdError:
        pass
