"""Baseline JPEG encode -- CPU restatement, test infrastructure only.

Reference interface replaced: the frame write of the hot
loop, ``cv2.imwrite(path, cv2.cvtColor(img, RGB2BGR))`` of every processed frame
(combine_detect.py:174-180, called at :259-262), which ``create_video`` then
reads back (:479-595). cv2 encodes through its bundled libjpeg-turbo [ext] with
quality 95 and 4:2:0 sampling; this restates libjpeg-turbo's compressor with its
defaults (Pillow 12.2 / libjpeg-turbo, importable here, runs the same code with
the same settings and pins it byte for byte: tests/test_jpeg_enc.py):

* ``rgb_ycc_convert`` (jccolor.c): 16-bit fixed-point tables, ONE_HALF rounding;
* edge expansion (jcprepct.c ``expand_bottom_edge``, jcsample.c
  ``expand_right_edge``): the last column / row replicated to whole blocks;
* ``h2v1_downsample`` / ``h2v2_downsample`` (jcsample.c): box average with the
  alternating bias 0,1 / 1,2;
* ``jpeg_fdct_islow`` (jfdctint.c: CONST_BITS 13, PASS1_BITS 2, output x8);
* ``quantize`` (jcdctmgr.c) through ``compute_reciprocal`` (16-bit DCTELEM of the
  SIMD build): q = sign(x) * (((|x| + corr) * recip) >> shift), which is what the
  AVX2 path computes;
* ``jpeg_set_quality`` (jcparam.c: Annex K tables, scale 200 - 2q / 5000 / q,
  baseline clamp to 255); ``std_huff_tables``; dummy blocks at the right /
  bottom MCU edge with the DC of their left / upper neighbour (jccoefct.c);
* ``encode_one_block`` (jchuff.c), 0xFF byte stuffing, 1-bit padding; JFIF 1.01
  APP0, DQT x2, SOF0, DHT x4, SOS markers in libjpeg's order.

Parity with cv2's header bytes is unpinned (cv2 is absent); the entropy-coded data
of a given quality and sampling is libjpeg-turbo's. Pure Python: small images only.
"""
import numpy as np

from oracle.jpeg import ZIGZAG

STD_LUMA = np.array([16, 11, 10, 16, 24, 40, 51, 61, 12, 12, 14, 19, 26, 58, 60, 55, 14, 13, 16, 24, 40, 57, 69, 56,
                     14, 17, 22, 29, 51, 87, 80, 62, 18, 22, 37, 56, 68, 109, 103, 77, 24, 35, 55, 64, 81, 104, 113,
                     92, 49, 64, 78, 87, 103, 121, 120, 101, 72, 92, 95, 98, 112, 100, 103, 99], np.int64)
STD_CHROMA = np.array([17, 18, 24, 47, 99, 99, 99, 99, 18, 21, 26, 66, 99, 99, 99, 99, 24, 26, 56, 99, 99, 99, 99, 99,
                       47, 66, 99, 99, 99, 99, 99, 99] + [99] * 32, np.int64)

# Annex K.3 tables: (bits[1..16], values)
DC_LUMA = ([0, 1, 5, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0], list(range(12)))
DC_CHROMA = ([0, 3, 1, 1, 1, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0], list(range(12)))
AC_LUMA = ([0, 2, 1, 3, 3, 2, 4, 3, 5, 5, 4, 4, 0, 0, 1, 0x7d], [
    0x01, 0x02, 0x03, 0x00, 0x04, 0x11, 0x05, 0x12, 0x21, 0x31, 0x41, 0x06, 0x13, 0x51, 0x61, 0x07, 0x22, 0x71, 0x14,
    0x32, 0x81, 0x91, 0xa1, 0x08, 0x23, 0x42, 0xb1, 0xc1, 0x15, 0x52, 0xd1, 0xf0, 0x24, 0x33, 0x62, 0x72, 0x82, 0x09,
    0x0a, 0x16, 0x17, 0x18, 0x19, 0x1a, 0x25, 0x26, 0x27, 0x28, 0x29, 0x2a, 0x34, 0x35, 0x36, 0x37, 0x38, 0x39, 0x3a,
    0x43, 0x44, 0x45, 0x46, 0x47, 0x48, 0x49, 0x4a, 0x53, 0x54, 0x55, 0x56, 0x57, 0x58, 0x59, 0x5a, 0x63, 0x64, 0x65,
    0x66, 0x67, 0x68, 0x69, 0x6a, 0x73, 0x74, 0x75, 0x76, 0x77, 0x78, 0x79, 0x7a, 0x83, 0x84, 0x85, 0x86, 0x87, 0x88,
    0x89, 0x8a, 0x92, 0x93, 0x94, 0x95, 0x96, 0x97, 0x98, 0x99, 0x9a, 0xa2, 0xa3, 0xa4, 0xa5, 0xa6, 0xa7, 0xa8, 0xa9,
    0xaa, 0xb2, 0xb3, 0xb4, 0xb5, 0xb6, 0xb7, 0xb8, 0xb9, 0xba, 0xc2, 0xc3, 0xc4, 0xc5, 0xc6, 0xc7, 0xc8, 0xc9, 0xca,
    0xd2, 0xd3, 0xd4, 0xd5, 0xd6, 0xd7, 0xd8, 0xd9, 0xda, 0xe1, 0xe2, 0xe3, 0xe4, 0xe5, 0xe6, 0xe7, 0xe8, 0xe9, 0xea,
    0xf1, 0xf2, 0xf3, 0xf4, 0xf5, 0xf6, 0xf7, 0xf8, 0xf9, 0xfa])
AC_CHROMA = ([0, 2, 1, 2, 4, 4, 3, 4, 7, 5, 4, 4, 0, 1, 2, 0x77], [
    0x00, 0x01, 0x02, 0x03, 0x11, 0x04, 0x05, 0x21, 0x31, 0x06, 0x12, 0x41, 0x51, 0x07, 0x61, 0x71, 0x13, 0x22, 0x32,
    0x81, 0x08, 0x14, 0x42, 0x91, 0xa1, 0xb1, 0xc1, 0x09, 0x23, 0x33, 0x52, 0xf0, 0x15, 0x62, 0x72, 0xd1, 0x0a, 0x16,
    0x24, 0x34, 0xe1, 0x25, 0xf1, 0x17, 0x18, 0x19, 0x1a, 0x26, 0x27, 0x28, 0x29, 0x2a, 0x35, 0x36, 0x37, 0x38, 0x39,
    0x3a, 0x43, 0x44, 0x45, 0x46, 0x47, 0x48, 0x49, 0x4a, 0x53, 0x54, 0x55, 0x56, 0x57, 0x58, 0x59, 0x5a, 0x63, 0x64,
    0x65, 0x66, 0x67, 0x68, 0x69, 0x6a, 0x73, 0x74, 0x75, 0x76, 0x77, 0x78, 0x79, 0x7a, 0x82, 0x83, 0x84, 0x85, 0x86,
    0x87, 0x88, 0x89, 0x8a, 0x92, 0x93, 0x94, 0x95, 0x96, 0x97, 0x98, 0x99, 0x9a, 0xa2, 0xa3, 0xa4, 0xa5, 0xa6, 0xa7,
    0xa8, 0xa9, 0xaa, 0xb2, 0xb3, 0xb4, 0xb5, 0xb6, 0xb7, 0xb8, 0xb9, 0xba, 0xc2, 0xc3, 0xc4, 0xc5, 0xc6, 0xc7, 0xc8,
    0xc9, 0xca, 0xd2, 0xd3, 0xd4, 0xd5, 0xd6, 0xd7, 0xd8, 0xd9, 0xda, 0xe2, 0xe3, 0xe4, 0xe5, 0xe6, 0xe7, 0xe8, 0xe9,
    0xea, 0xf2, 0xf3, 0xf4, 0xf5, 0xf6, 0xf7, 0xf8, 0xf9, 0xfa])

SAMPLING = {0: (1, 1), 1: (2, 1), 2: (2, 2)}   # Pillow's subsampling -> luma (h, v); chroma is 1x1


def quant_table(std, quality):
    """jpeg_set_quality -> jpeg_quality_scaling + jpeg_add_quant_table(force_baseline)."""
    q = max(1, min(100, quality))
    scale = 5000 // q if q < 50 else 200 - 2 * q
    t = (std * scale + 50) // 100
    return np.clip(t, 1, 255)


def reciprocal(divisor):
    """compute_reciprocal (jcdctmgr.c) for a 16-bit DCTELEM: (recip, corr, shift)."""
    b = int(divisor).bit_length() - 1
    r = 16 + b
    fq, fr = divmod(1 << r, divisor)
    c = divisor // 2
    if fr == 0:
        fq >>= 1
        r -= 1
    elif fr <= divisor // 2:
        c += 1
    else:
        fq += 1
    return fq, c, r


def quantize(ws, q):
    """ws: [..., 64] FDCT output (natural order); q: [64] quant table -> coefficients."""
    out = np.empty_like(ws)
    for i in range(64):
        fq, c, r = reciprocal(int(q[i]) << 3)
        x = ws[..., i]
        m = ((np.abs(x) + c) * fq) >> r
        out[..., i] = np.where(x < 0, -m, m)
    return out


def rgb_ycc(rgb):
    """jccolor.c rgb_ycc_convert with its tables."""
    fix = lambda x: int(x * 65536 + 0.5)
    r, g, b = (rgb[..., i].astype(np.int64) for i in range(3))
    half, off = 1 << 15, 128 << 16
    y = (fix(0.29900) * r + fix(0.58700) * g + fix(0.11400) * b + half) >> 16
    cb = (-fix(0.16874) * r - fix(0.33126) * g + fix(0.5) * b + off + half - 1) >> 16
    cr = (fix(0.5) * r - fix(0.41869) * g - fix(0.08131) * b + off + half - 1) >> 16
    return y, cb, cr


def _pad(p, h, w):
    """Replicate the last row / column up to h x w (expand_bottom/right_edge)."""
    return np.pad(p, ((0, h - p.shape[0]), (0, w - p.shape[1])), mode="edge")


def downsample(p, hs, vs, oh, ow):
    """h2v2 / h2v1 box average with libjpeg's alternating bias; p already padded to
    (oh * vs) x (ow * hs)."""
    if hs == 1 and vs == 1:
        return p[:oh, :ow]
    if hs == 2 and vs == 1:
        bias = np.tile([0, 1], ow // 2 + 1)[:ow]
        return (p[:oh, 0:2 * ow:2] + p[:oh, 1:2 * ow:2] + bias) >> 1
    bias = np.tile([1, 2], ow // 2 + 1)[:ow]
    return (p[0:2 * oh:2, 0:2 * ow:2] + p[0:2 * oh:2, 1:2 * ow:2] + p[1:2 * oh:2, 0:2 * ow:2] +
            p[1:2 * oh:2, 1:2 * ow:2] + bias) >> 2


F = dict(f0298=2446, f0390=3196, f0541=4433, f0765=6270, f0899=7373, f1175=9633, f1501=12299, f1847=15137,
         f1961=16069, f2053=16819, f2562=20995, f3072=25172)


def _desc(x, n):
    return (x + (1 << (n - 1))) >> n


def _fdct_1d(d, first):
    """One jpeg_fdct_islow pass over axis -1 (8 samples)."""
    d0, d1, d2, d3, d4, d5, d6, d7 = (d[..., i] for i in range(8))
    t0, t7 = d0 + d7, d0 - d7
    t1, t6 = d1 + d6, d1 - d6
    t2, t5 = d2 + d5, d2 - d5
    t3, t4 = d3 + d4, d3 - d4
    t10, t13 = t0 + t3, t0 - t3
    t11, t12 = t1 + t2, t1 - t2
    o = np.empty_like(d)
    sh = 13 - 2 if first else 13 + 2
    if first:
        o[..., 0] = (t10 + t11) << 2
        o[..., 4] = (t10 - t11) << 2
    else:
        o[..., 0] = _desc(t10 + t11, 2)
        o[..., 4] = _desc(t10 - t11, 2)
    z1 = (t12 + t13) * F["f0541"]
    o[..., 2] = _desc(z1 + t13 * F["f0765"], sh)
    o[..., 6] = _desc(z1 - t12 * F["f1847"], sh)
    z1, z2, z3, z4 = t4 + t7, t5 + t6, t4 + t6, t5 + t7
    z5 = (z3 + z4) * F["f1175"]
    t4, t5, t6, t7 = t4 * F["f0298"], t5 * F["f2053"], t6 * F["f3072"], t7 * F["f1501"]
    z1, z2, z3, z4 = -z1 * F["f0899"], -z2 * F["f2562"], -z3 * F["f1961"], -z4 * F["f0390"]
    z3 = z3 + z5
    z4 = z4 + z5
    o[..., 7] = _desc(t4 + z1 + z3, sh)
    o[..., 5] = _desc(t5 + z2 + z4, sh)
    o[..., 3] = _desc(t6 + z2 + z3, sh)
    o[..., 1] = _desc(t7 + z1 + z4, sh)
    return o


def fdct_islow(blocks):
    """blocks: [..., 8, 8] int64 samples - 128 -> [..., 8, 8] (scaled by 8)."""
    r = _fdct_1d(blocks, True)                                   # rows
    c = _fdct_1d(np.swapaxes(r, -1, -2), False)                  # columns
    return np.swapaxes(c, -1, -2)


def component_blocks(rgb, sub=2, quality=95):
    """Quantized coefficient blocks per component, natural order:
    list of [bh, bw, 64] (the component's real blocks, width/height_in_blocks)."""
    h, w, _ = rgb.shape
    hl, vl = SAMPLING[sub]
    y, cb, cr = rgb_ycc(rgb)
    out = []
    for ci, p in enumerate((y, cb, cr)):
        hs, vs = (hl, vl) if ci == 0 else (1, 1)
        bw, bh = -(-w * hs // (hl * 8)), -(-h * vs // (vl * 8))     # width/height_in_blocks
        if ci == 0:
            s = _pad(p, bh * 8, bw * 8)
        else:
            # full-res rows to the end of the last row group and columns to the block edge
            # replicated (color_buf / expand_right_edge), box average, then the last
            # downsampled row replicated to whole blocks (expand_bottom_edge of output_buf)
            rows = -(-h // vl)
            ds = downsample(_pad(p, rows * vl, bw * 8 * hl), hl, vl, rows, bw * 8)
            s = _pad(ds, bh * 8, bw * 8)
        blk = s.reshape(bh, 8, bw, 8).swapaxes(1, 2) - 128
        coef = fdct_islow(blk).reshape(bh, bw, 64)
        q = quant_table(STD_LUMA if ci == 0 else STD_CHROMA, quality)
        out.append(quantize(coef, q))
    return out


class _BitWriter:
    def __init__(self):
        self.out = bytearray()
        self.acc = 0
        self.n = 0

    def put(self, code, size):
        self.acc = (self.acc << size) | (code & ((1 << size) - 1))
        self.n += size
        while self.n >= 8:
            self.n -= 8
            byte = (self.acc >> self.n) & 0xFF
            self.out.append(byte)
            if byte == 0xFF:
                self.out.append(0)

    def flush(self):
        """flush_bits (jchuff.c): seven 1-bits fill the partial byte, the rest is dropped."""
        self.put(0x7F, 7)
        self.acc = self.n = 0


def _codes(tab):
    bits, vals = tab
    codes, code, k = {}, 0, 0
    for ln in range(1, 17):
        for _ in range(bits[ln - 1]):
            codes[vals[k]] = (code, ln)
            code += 1
            k += 1
        code <<= 1
    return codes


def _nbits(v):
    return int(abs(int(v))).bit_length()


def _encode_block(bw, zz, last_dc, dc, ac):
    diff = int(zz[0]) - last_dc
    nb = _nbits(diff)
    bw.put(*dc[nb])
    if nb:
        bw.put(diff if diff >= 0 else diff - 1, nb)
    r = 0
    for k in range(1, 64):
        v = int(zz[k])
        if v == 0:
            r += 1
            continue
        while r > 15:
            bw.put(*ac[0xF0])
            r -= 16
        nb = _nbits(v)
        bw.put(*ac[(r << 4) + nb])
        bw.put(v if v >= 0 else v - 1, nb)
        r = 0
    if r:
        bw.put(*ac[0x00])
    return int(zz[0])


def _marker_dht(tc, th, tab):
    bits, vals = tab
    body = bytes([tc << 4 | th]) + bytes(bits) + bytes(vals)
    return b"\xff\xc4" + (len(body) + 2).to_bytes(2, "big") + body


def encode(rgb, quality=95, sub=2):
    """uint8 [h, w, 3] RGB -> JFIF bytes, byte-identical to Pillow's
    Image.save(..., "JPEG", quality=quality, subsampling=sub)."""
    h, w, _ = rgb.shape
    hl, vl = SAMPLING[sub]
    comps = component_blocks(rgb, sub, quality)
    ql, qc = quant_table(STD_LUMA, quality), quant_table(STD_CHROMA, quality)
    out = bytearray(b"\xff\xd8")
    out += b"\xff\xe0\x00\x10JFIF\x00\x01\x01\x00\x00\x01\x00\x01\x00\x00"
    for t, q in ((0, ql), (1, qc)):
        out += b"\xff\xdb\x00\x43" + bytes([t]) + bytes(int(v) for v in q[ZIGZAG])
    out += b"\xff\xc0\x00\x11\x08" + h.to_bytes(2, "big") + w.to_bytes(2, "big") + b"\x03"
    out += bytes([1, hl << 4 | vl, 0, 2, 0x11, 1, 3, 0x11, 1])
    out += _marker_dht(0, 0, DC_LUMA) + _marker_dht(1, 0, AC_LUMA) + _marker_dht(0, 1, DC_CHROMA) + \
        _marker_dht(1, 1, AC_CHROMA)
    out += b"\xff\xda\x00\x0c\x03\x01\x00\x02\x11\x03\x11\x00\x3f\x00"
    tabs = [(_codes(DC_LUMA), _codes(AC_LUMA)), (_codes(DC_CHROMA), _codes(AC_CHROMA))]
    bw = _BitWriter()
    last = [0, 0, 0]
    mcux, mcuy = -(-w // (8 * hl)), -(-h // (8 * vl))
    zz = [c[..., ZIGZAG] for c in comps]                      # natural -> zigzag order
    for my in range(mcuy):
        for mx in range(mcux):
            for ci in range(3):
                hs, vs = (hl, vl) if ci == 0 else (1, 1)
                dc, ac = tabs[0 if ci == 0 else 1]
                bh, bwid = zz[ci].shape[:2]
                prev = None
                for yy in range(vs):
                    row_dc = None
                    for xx in range(hs):
                        by, bx = my * vs + yy, mx * hs + xx
                        if by < bh and bx < bwid:
                            blk = zz[ci][by, bx]
                        else:                       # dummy block: zero AC, DC of its left / upper neighbour
                            blk = np.zeros(64, np.int64)
                            blk[0] = row_dc if (by < bh and row_dc is not None) else prev
                        last[ci] = _encode_block(bw, blk, last[ci], dc, ac)
                        row_dc = int(blk[0])
                        prev = int(blk[0])
    bw.flush()
    out += bw.out
    out += b"\xff\xd9"
    return bytes(out)
