"""Baseline JPEG decode -- CPU restatement, test infrastructure only.

Reference interface replaced: the frame I/O around the hot
path -- ffmpeg-split JPEG frames read by ``cv2.imread`` + BGR->RGB
(combine_detect.py:167-172) in ``batch_process_images`` (:183-277). cv2 decodes
through its bundled libjpeg-turbo [ext] with the library defaults, which this
restates (Pillow 12.2 / libjpeg-turbo "jpeg 6.2" API, importable here, decodes with
the same defaults and pins it: tests/test_jpeg.py):

* entropy decode: baseline sequential Huffman (ITU T.81 F.2.2), restart markers;
* dequantize + ``jpeg_idct_islow`` (jidctint.c: CONST_BITS 13, PASS1_BITS 2, the
  LL&M 12-multiply integer IDCT, ``range_limit`` post-IDCT table incl. its
  ``& RANGE_MASK`` wrap);
* ``do_fancy_upsampling`` (default TRUE): h2v1 / h2v2 triangle filters of
  jdsample.c, edge rows/columns replicated (jdmainct.c context rows);
* ``ycc_rgb_convert`` (jdcolor.c): 16-bit fixed-point tables, ``range_limit``.

Parity with cv2 itself is unpinned (cv2 is absent here); cv2 and Pillow both use
libjpeg-turbo's default decode path. Pure Python: small images only.
"""
import numpy as np

ZIGZAG = np.array([0, 1, 8, 16, 9, 2, 3, 10, 17, 24, 32, 25, 18, 11, 4, 5, 12, 19, 26, 33, 40, 48, 41, 34, 27, 20,
                   13, 6, 7, 14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51, 58, 59, 52,
                   45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63], np.int64)   # zigzag k -> natural index


class Jpeg:
    def __init__(self):
        self.q = {}
        self.huff = {}
        self.comps = []
        self.h = self.w = 0
        self.restart = 0


def _u16(b, o):
    return (b[o] << 8) | b[o + 1]


def parse(data):
    """Markers -> Jpeg with tables, frame header, and the entropy-coded segment."""
    b = memoryview(data)
    if b[0] != 0xFF or b[1] != 0xD8:
        raise ValueError("not a JPEG (no SOI)")
    j = Jpeg()
    o = 2
    while o < len(b):
        while b[o] == 0xFF and b[o + 1] == 0xFF:
            o += 1
        if b[o] != 0xFF:
            raise ValueError("marker expected")
        m = b[o + 1]
        o += 2
        if m == 0xD9:
            break
        ln = _u16(b, o)
        seg = bytes(b[o + 2:o + ln])
        if m == 0xDB:                                   # DQT
            p = 0
            while p < len(seg):
                pq, tq = seg[p] >> 4, seg[p] & 15
                p += 1
                n = 64 * (2 if pq else 1)
                vals = np.frombuffer(seg[p:p + n], ">u2" if pq else "u1").astype(np.int64)
                q = np.zeros(64, np.int64)
                q[ZIGZAG] = vals                        # stored in zigzag order
                j.q[tq] = q
                p += n
        elif m == 0xC4:                                 # DHT
            p = 0
            while p < len(seg):
                tc, th = seg[p] >> 4, seg[p] & 15
                counts = list(seg[p + 1:p + 17])
                p += 17
                syms = list(seg[p:p + sum(counts)])
                p += sum(counts)
                codes = {}
                code, k = 0, 0
                for ln_ in range(1, 17):
                    for _ in range(counts[ln_ - 1]):
                        codes[(ln_, code)] = syms[k]
                        k += 1
                        code += 1
                    code <<= 1
                j.huff[(tc, th)] = codes
        elif m in (0xC0, 0xC1):                         # SOF0 / SOF1 (baseline / extended Huffman)
            if seg[0] != 8:
                raise ValueError("only 8-bit samples")
            j.h, j.w = _u16(seg, 1), _u16(seg, 3)
            nc = seg[5]
            j.comps = [dict(id=seg[6 + 3 * i], hs=seg[7 + 3 * i] >> 4, vs=seg[7 + 3 * i] & 15, tq=seg[8 + 3 * i])
                       for i in range(nc)]
        elif m in (0xC2, 0xC3, 0xC5, 0xC6, 0xC7, 0xC9, 0xCA, 0xCB, 0xCD, 0xCE, 0xCF):
            raise ValueError("progressive / lossless / arithmetic JPEG not supported")
        elif m == 0xDD:                                 # DRI
            j.restart = _u16(seg, 0)
        elif m == 0xDA:                                 # SOS: entropy data follows
            ns = seg[0]
            ids = [seg[1 + 2 * i] for i in range(ns)]
            tabs = [(seg[2 + 2 * i] >> 4, seg[2 + 2 * i] & 15) for i in range(ns)]
            if ns != len(j.comps):
                raise ValueError("non-interleaved scans not supported")
            for c, i_, t in zip(j.comps, ids, tabs):
                assert c["id"] == i_
                c["td"], c["ta"] = t
            o += ln
            end = o
            while True:                                 # entropy segment ends at a non-RST marker
                if b[end] == 0xFF and b[end + 1] != 0x00 and not (0xD0 <= b[end + 1] <= 0xD7):
                    break
                end += 1
            j.scan = bytes(b[o:end])
            o = end
            continue
        o += ln
    return j


class _Bits:
    def __init__(self, data):
        self.d = data
        self.p = 0
        self.acc = 0
        self.n = 0

    def _byte(self):
        if self.p >= len(self.d):
            return 0                                   # pad with zeros past the end (libjpeg does too)
        v = self.d[self.p]
        self.p += 1
        if v == 0xFF:
            nxt = self.d[self.p] if self.p < len(self.d) else 0
            if nxt == 0x00:
                self.p += 1
            else:                                      # a marker: do not consume, feed zeros
                self.p -= 1
                return 0
        return v

    def bit(self):
        if self.n == 0:
            self.acc = self._byte()
            self.n = 8
        self.n -= 1
        return (self.acc >> self.n) & 1

    def bits(self, k):
        v = 0
        for _ in range(k):
            v = (v << 1) | self.bit()
        return v

    def restart(self):
        self.n = 0
        while self.p + 1 < len(self.d) and not (self.d[self.p] == 0xFF and 0xD0 <= self.d[self.p + 1] <= 0xD7):
            self.p += 1
        self.p += 2


def _decode_sym(bits, codes):
    code, ln = 0, 0
    while ln < 16:
        code = (code << 1) | bits.bit()
        ln += 1
        if (ln, code) in codes:
            return codes[(ln, code)]
    raise ValueError("bad Huffman code")


def _extend(v, s):
    return v - (1 << s) + 1 if s and v < (1 << (s - 1)) else v


def coefficients(j):
    """Entropy decode -> per component int64 [blocks_h][blocks_w][64] (natural order,
    quantized), over the MCU-padded component size."""
    hmax = max(c["hs"] for c in j.comps)
    vmax = max(c["vs"] for c in j.comps)
    mcux = -(-j.w // (8 * hmax))
    mcuy = -(-j.h // (8 * vmax))
    out = [np.zeros((mcuy * c["vs"], mcux * c["hs"], 64), np.int64) for c in j.comps]
    bits = _Bits(j.scan)
    pred = [0] * len(j.comps)
    n = 0
    for my in range(mcuy):
        for mx in range(mcux):
            if j.restart and n and n % j.restart == 0:
                bits.restart()
                pred = [0] * len(j.comps)
            n += 1
            for ci, c in enumerate(j.comps):
                dc, ac = j.huff[(0, c["td"])], j.huff[(1, c["ta"])]
                for by in range(c["vs"]):
                    for bx in range(c["hs"]):
                        blk = out[ci][my * c["vs"] + by, mx * c["hs"] + bx]
                        s = _decode_sym(bits, dc)
                        pred[ci] += _extend(bits.bits(s), s)
                        blk[0] = pred[ci]
                        k = 1
                        while k < 64:
                            rs = _decode_sym(bits, ac)
                            r, s = rs >> 4, rs & 15
                            if s == 0:
                                if r != 15:
                                    break
                                k += 16
                                continue
                            k += r
                            blk[ZIGZAG[k]] = _extend(bits.bits(s), s)
                            k += 1
    return out


CONST_BITS, PASS1_BITS = 13, 2
F = {n: v for n, v in [("0_298631336", 2446), ("0_390180644", 3196), ("0_541196100", 4433), ("0_765366865", 6270),
                       ("0_899976223", 7373), ("1_175875602", 9633), ("1_501321110", 12299),
                       ("1_847759065", 15137), ("1_961570560", 16069), ("2_053119869", 16819),
                       ("2_562915447", 20995), ("3_072711026", 25172)]}


def _range_limit_idct(x):
    """range_limit[x & RANGE_MASK] of the post-IDCT table (jdmaster.c prepare_range_limit_table)."""
    j = x & 1023
    return np.where(j < 128, j + 128, np.where(j < 512, 255, np.where(j < 896, 0, j - 896))).astype(np.uint8)


def idct_islow(coef, q):
    """jidctint.c jpeg_idct_islow on blocks [..., 64] (natural order) -> uint8 [..., 8, 8]."""
    c = (coef * q).reshape(coef.shape[:-1] + (8, 8)).astype(np.int64)   # [.., row u, col v]

    def one_d(z0, z1, z2, z3, z4, z5, z6, z7, first):
        # even part
        if first:
            z2e, z3e = z2, z6
            zz = (z2e + z3e) * F["0_541196100"]
            tmp2 = zz + z3e * (-F["1_847759065"])
            tmp3 = zz + z2e * F["0_765366865"]
            tmp0 = (z0 + z4) << CONST_BITS
            tmp1 = (z0 - z4) << CONST_BITS
        else:
            z2e, z3e = z2, z6
            zz = (z2e + z3e) * F["0_541196100"]
            tmp2 = zz + z3e * (-F["1_847759065"])
            tmp3 = zz + z2e * F["0_765366865"]
            tmp0 = (z0 + z4) << CONST_BITS
            tmp1 = (z0 - z4) << CONST_BITS
        tmp10, tmp13 = tmp0 + tmp3, tmp0 - tmp3
        tmp11, tmp12 = tmp1 + tmp2, tmp1 - tmp2
        # odd part
        t0, t1, t2, t3 = z7, z5, z3, z1
        za, zb, zc, zd = t0 + t3, t1 + t2, t0 + t2, t1 + t3
        z5_ = (zc + zd) * F["1_175875602"]
        t0 = t0 * F["0_298631336"]
        t1 = t1 * F["2_053119869"]
        t2 = t2 * F["3_072711026"]
        t3 = t3 * F["1_501321110"]
        za = za * (-F["0_899976223"])
        zb = zb * (-F["2_562915447"])
        zc = zc * (-F["1_961570560"]) + z5_
        zd = zd * (-F["0_390180644"]) + z5_
        t0 += za + zc
        t1 += zb + zd
        t2 += zb + zc
        t3 += za + zd
        return [tmp10 + t3, tmp11 + t2, tmp12 + t1, tmp13 + t0, tmp13 - t0, tmp12 - t1, tmp11 - t2, tmp10 - t3]

    # pass 1: columns (input rows u = 0..7 of column v), descale by CONST_BITS - PASS1_BITS
    cols = [c[..., u, :] for u in range(8)]                # each [..., 8 columns]
    o = one_d(*cols, first=True)
    ws = np.stack([(v + (1 << (CONST_BITS - PASS1_BITS - 1))) >> (CONST_BITS - PASS1_BITS) for v in o], -2)
    # pass 2: rows; libjpeg-turbo folds the rounding into the DC term
    rows = [ws[..., :, v] for v in range(8)]               # each [..., 8 rows]
    rows[0] = rows[0] + (1 << (PASS1_BITS + 2))
    o = one_d(*rows, first=False)
    out = np.stack([_range_limit_idct(v >> (CONST_BITS + PASS1_BITS + 3)) for v in o], -1)
    return out


def planes(j, coefs):
    """Per component the decoded sample plane [blocks_h*8][blocks_w*8] uint8."""
    res = []
    for c, cf in zip(j.comps, coefs):
        blk = idct_islow(cf, j.q[c["tq"]])                 # [bh][bw][8][8]
        bh, bw = blk.shape[:2]
        res.append(blk.transpose(0, 2, 1, 3).reshape(bh * 8, bw * 8))
    return res


def upsample_fancy(p, hs, vs, dw, dh, w, h):
    """jdsample.c fancy upsampling of a downsampled plane (valid size dw x dh) to w x h."""
    x = p[:dh, :dw].astype(np.int64)
    if hs == 1 and vs == 1:
        return x[:h, :w]
    if hs == 2 and vs == 1:                                # h2v1
        left = np.concatenate([x[:, :1], x[:, :-1]], 1)
        right = np.concatenate([x[:, 1:], x[:, -1:]], 1)
        even = (x * 3 + left + 1) >> 2
        odd = (x * 3 + right + 2) >> 2
        even[:, 0] = x[:, 0]
        odd[:, -1] = x[:, -1]
        out = np.stack([even, odd], 2).reshape(x.shape[0], -1)
        return out[:h, :w].astype(np.uint8)
    if hs == 2 and vs == 2:                                # h2v2
        up = np.concatenate([x[:1], x[:-1]], 0)            # row above (top row replicated)
        dn = np.concatenate([x[1:], x[-1:]], 0)            # row below (last row replicated)
        rows = []
        for nb in (up, dn):                                # v = 0: nearer row above, v = 1: below
            cs = x * 3 + nb                                # column sums
            last = np.concatenate([cs[:, :1], cs[:, :-1]], 1)
            nxt = np.concatenate([cs[:, 1:], cs[:, -1:]], 1)
            even = (cs * 3 + last + 8) >> 4
            odd = (cs * 3 + nxt + 7) >> 4
            even[:, 0] = (cs[:, 0] * 4 + 8) >> 4
            odd[:, -1] = (cs[:, -1] * 4 + 7) >> 4
            rows.append(np.stack([even, odd], 2).reshape(x.shape[0], -1))
        out = np.stack(rows, 1).reshape(-1, rows[0].shape[1])
        return out[:h, :w].astype(np.uint8)
    raise ValueError(f"sampling {hs}x{vs} not supported")


SCALEBITS = 16
ONE_HALF = 1 << (SCALEBITS - 1)


def _fix(x):
    return int(x * (1 << SCALEBITS) + 0.5)


def ycc_rgb(y, cb, cr):
    """jdcolor.c ycc_rgb_convert (build_ycc_rgb_table), range_limit clamps."""
    x = np.arange(256) - 128
    cr_r = (_fix(1.40200) * x + ONE_HALF) >> SCALEBITS
    cb_b = (_fix(1.77200) * x + ONE_HALF) >> SCALEBITS
    cr_g = -_fix(0.71414) * x
    cb_g = -_fix(0.34414) * x + ONE_HALF
    y = y.astype(np.int64)
    r = y + cr_r[cr]
    g = y + ((cb_g[cb] + cr_g[cr]) >> SCALEBITS)
    b = y + cb_b[cb]
    return np.stack([np.clip(r, 0, 255), np.clip(g, 0, 255), np.clip(b, 0, 255)], -1).astype(np.uint8)


def decode(data):
    """JPEG bytes -> uint8 RGB [h][w][3] (grayscale -> replicated)."""
    j = parse(data)
    coefs = coefficients(j)
    pl = planes(j, coefs)
    hmax = max(c["hs"] for c in j.comps)
    vmax = max(c["vs"] for c in j.comps)
    up = []
    for c, p in zip(j.comps, pl):
        dw = -(-j.w * c["hs"] // hmax)
        dh = -(-j.h * c["vs"] // vmax)
        up.append(upsample_fancy(p, hmax // c["hs"], vmax // c["vs"], dw, dh, j.w, j.h))
    if len(up) == 1:
        return np.repeat(up[0][..., None], 3, -1)
    return ycc_rgb(up[0], up[1], up[2])
