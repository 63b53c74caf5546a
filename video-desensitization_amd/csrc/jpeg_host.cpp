// jpeg_host.cpp — baseline JPEG frame decode: host entropy stage + C-ABI.
//
// Replaces the frame read of the reference's hot loop: the ffmpeg-split JPEG
// frames (combine_detect.py:279-476) read by cv2.imread + BGR->RGB
// (combine_detect.py:167-172) inside batch_process_images (:183-277). cv2 decodes
// with its libjpeg-turbo [ext] defaults: ISLOW IDCT, fancy upsampling, table-based
// YCbCr->RGB; the result here is bit-identical (oracle/jpeg.py, pinned against
// Pillow's libjpeg-turbo; tests/test_jpeg.py).
//
// Split of the work:
//   host (this file)  marker parse + Huffman entropy decode (bit-serial, one image
//                     per thread) into a sparse coefficient stream: per block an
//                     offset, per nonzero coefficient one u32 (natural index << 16 |
//                     int16 value); ~10 entries per block at q95, a fraction of the
//                     6.2 MB a dense 1080p coefficient image would cross PCIe with;
//   device (jpeg.hip) dequantize + ISLOW IDCT per block, fancy upsampling +
//                     YCbCr->RGB per pixel, straight into the frame batch that
//                     vd_process reads (no host RGB frame, no second H2D).
#include "../../include/vdmi.h"
#include "vd_common.h"
#include "nets.h"

#include <algorithm>
#include <atomic>
#include <cstring>
#include <thread>
#include <memory>
#include <vector>

namespace {

const int kZigzag[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48,
                         41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23,
                         30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

constexpr int kLook = 11;                 // lookahead bits

struct Huff {
    // kLook-bit lookahead: len 0 = longer code (slow path)
    uint8_t look_len[1 << kLook];
    uint8_t look_sym[1 << kLook];
    // AC fast path (libjpeg-turbo style): code AND its extra bits inside the window
    // -> total bits, coefficient run and value; len 0 = not decodable in one look
    uint8_t fa_len[1 << kLook];
    uint8_t fa_run[1 << kLook];              // k advance: r (value), 16 (ZRL), 64 (EOB)
    int16_t fa_val[1 << kLook];
    int32_t maxcode[18];      // largest code of length l (-1 if none), maxcode[17] sentinel
    int32_t valoff[17];       // symbol index of the first code of length l minus that code
    uint8_t vals[256];
    bool present = false;
};

struct Comp { int id = -1, hs = 0, vs = 0, tq = 0, td = 0, ta = 0, bw = 0, bh = 0; bool scanned = false; };

struct Info {
    int h = 0, w = 0, nc = 0, hmax = 1, vmax = 1, mcux = 0, mcuy = 0, restart = 0;
    Comp c[3];
    uint16_t q[4][64];        // natural order
    bool qpresent[4] = {false, false, false, false};
    Huff dc[4], ac[4];
    const uint8_t* scan = nullptr;
    size_t scan_len = 0;
};

int build_huff(Huff& hf, const uint8_t* counts, const uint8_t* syms, int nsym) {
    if (nsym > 256) return -1;
    memcpy(hf.vals, syms, nsym);
    memset(hf.look_len, 0, sizeof hf.look_len);
    memset(hf.fa_len, 0, sizeof hf.fa_len);
    int code = 0, k = 0;
    for (int l = 1; l <= 16; ++l) {
        hf.valoff[l] = k - code;
        for (int i = 0; i < counts[l - 1]; ++i, ++k, ++code) {
            // an over-subscribed table would index past the lookahead arrays below:
            // reject it before any fill (code must fit in l bits)
            if (code >= (1 << l)) return -1;
            if (l <= kLook) {   // fill every kLook-bit prefix extension
                const int base = code << (kLook - l);
                const int rs = syms[k], r = rs >> 4, sz = rs & 15;
                for (int e = 0; e < (1 << (kLook - l)); ++e) {
                    hf.look_len[base + e] = (uint8_t)l;
                    hf.look_sym[base + e] = syms[k];
                    if (sz == 0) {                       // EOB / ZRL (AC tables)
                        hf.fa_len[base + e] = (uint8_t)l;
                        hf.fa_run[base + e] = r == 15 ? 16 : 64;
                        hf.fa_val[base + e] = 0;
                    } else if (l + sz <= kLook) {
                        const int extra = (e >> (kLook - l - sz)) & ((1 << sz) - 1);
                        hf.fa_len[base + e] = (uint8_t)(l + sz);
                        hf.fa_run[base + e] = (uint8_t)r;
                        hf.fa_val[base + e] = (int16_t)(extra < (1 << (sz - 1)) ? extra - (1 << sz) + 1 : extra);
                    }
                }
            }
        }
        hf.maxcode[l] = counts[l - 1] ? code - 1 : -1;
        code <<= 1;
    }
    hf.maxcode[17] = 0x7fffffff;
    hf.present = true;
    return 0;
}

inline int u16be(const uint8_t* p) { return (p[0] << 8) | p[1]; }

// header_only: stop at the scan header (frame size / layout known, the entropy-coded
// segment neither delimited nor checked): what vd_jpeg_info needs
int parse(const uint8_t* d, size_t n, Info& j, bool header_only = false) {
    if (n < 4 || d[0] != 0xFF || d[1] != 0xD8) return vd_set_error(VD_ERR_ARG, "jpeg: no SOI marker");
    size_t o = 2;
    bool sof = false;
    while (o + 4 <= n) {
        if (d[o] != 0xFF) return vd_set_error(VD_ERR_ARG, "jpeg: marker expected at %zu", o);
        while (o + 1 < n && d[o + 1] == 0xFF) ++o;
        const int m = d[o + 1];
        o += 2;
        if (m == 0xD9) break;
        if (o + 2 > n) break;
        const int len = u16be(d + o);
        if (len < 2 || o + len > n) return vd_set_error(VD_ERR_ARG, "jpeg: truncated segment 0x%02X", m);
        const uint8_t* s = d + o + 2;
        const int sl = len - 2;
        if (m == 0xDB) {                                   // DQT
            int p = 0;
            while (p < sl) {
                const int pq = s[p] >> 4, tq = s[p] & 15;
                ++p;
                if (tq > 3 || p + 64 * (pq ? 2 : 1) > sl) return vd_set_error(VD_ERR_ARG, "jpeg: bad DQT");
                for (int k = 0; k < 64; ++k) {
                    const int v = pq ? u16be(s + p + 2 * k) : s[p + k];
                    j.q[tq][kZigzag[k]] = (uint16_t)v;
                }
                j.qpresent[tq] = true;
                p += 64 * (pq ? 2 : 1);
            }
        } else if (m == 0xC4) {                            // DHT
            int p = 0;
            while (p + 17 <= sl) {
                const int tc = s[p] >> 4, th = s[p] & 15;
                const uint8_t* counts = s + p + 1;
                int ns = 0;
                for (int l = 0; l < 16; ++l) ns += counts[l];
                if (th > 3 || tc > 1 || p + 17 + ns > sl) return vd_set_error(VD_ERR_ARG, "jpeg: bad DHT");
                if (build_huff(tc ? j.ac[th] : j.dc[th], counts, s + p + 17, ns))
                    return vd_set_error(VD_ERR_ARG, "jpeg: bad Huffman table");
                p += 17 + ns;
            }
        } else if (m == 0xC0 || m == 0xC1) {               // SOF0 / SOF1
            if (sof) return vd_set_error(VD_ERR_ARG, "jpeg: more than one frame header");
            if (sl < 6 || s[0] != 8) return vd_set_error(VD_ERR_ARG, "jpeg: only 8-bit samples are supported");
            j.h = u16be(s + 1);
            j.w = u16be(s + 3);
            j.nc = s[5];
            if ((j.nc != 1 && j.nc != 3) || sl < 6 + 3 * j.nc || j.h <= 0 || j.w <= 0)
                return vd_set_error(VD_ERR_ARG, "jpeg: unsupported frame header (%d components)", j.nc);
            for (int i = 0; i < j.nc; ++i) {
                Comp& c = j.c[i];
                c.id = s[6 + 3 * i];
                c.hs = s[7 + 3 * i] >> 4;
                c.vs = s[7 + 3 * i] & 15;
                c.tq = s[8 + 3 * i] & 3;
                if (c.hs < 1 || c.hs > 2 || c.vs < 1 || c.vs > 2)
                    return vd_set_error(VD_ERR_ARG, "jpeg: sampling %dx%d not supported", c.hs, c.vs);
                for (int k = 0; k < i; ++k)
                    if (j.c[k].id == c.id) return vd_set_error(VD_ERR_ARG, "jpeg: duplicate component id %d", c.id);
            }
            sof = true;
        } else if ((m >= 0xC2 && m <= 0xCF) && m != 0xC4 && m != 0xC8 && m != 0xCC) {
            return vd_set_error(VD_ERR_ARG, "jpeg: progressive / lossless / arithmetic coding not supported");
        } else if (m == 0xDD) {                            // DRI
            if (sl < 2) return vd_set_error(VD_ERR_ARG, "jpeg: bad DRI");
            j.restart = u16be(s);
        } else if (m == 0xDA) {                            // SOS
            if (!sof) return vd_set_error(VD_ERR_ARG, "jpeg: SOS before SOF");
            if (j.scan) return vd_set_error(VD_ERR_ARG, "jpeg: more than one scan (not baseline)");
            if (sl < 1) return vd_set_error(VD_ERR_ARG, "jpeg: bad SOS");
            const int ns = s[0];
            if (ns != j.nc) return vd_set_error(VD_ERR_ARG, "jpeg: non-interleaved scans not supported");
            if (sl < 1 + 2 * ns + 3) return vd_set_error(VD_ERR_ARG, "jpeg: truncated SOS");
            for (int i = 0; i < ns; ++i) {
                const int id = s[1 + 2 * i];
                int ci = -1;
                for (int k = 0; k < j.nc; ++k) if (j.c[k].id == id) ci = k;
                if (ci < 0) return vd_set_error(VD_ERR_ARG, "jpeg: scan names an unknown component");
                if (j.c[ci].scanned) return vd_set_error(VD_ERR_ARG, "jpeg: scan names component %d twice", id);
                j.c[ci].scanned = true;
                j.c[ci].td = s[2 + 2 * i] >> 4;
                j.c[ci].ta = s[2 + 2 * i] & 15;
                if (j.c[ci].td > 3 || j.c[ci].ta > 3) return vd_set_error(VD_ERR_ARG, "jpeg: bad table index");
            }
            o += len;
            j.scan = d + o;
            if (header_only) return VD_OK;
            // the segment ends at the first marker that is neither a stuffed 0xFF00 nor RSTn:
            // memchr to each 0xFF instead of a byte loop
            size_t e = o;
            while (e + 1 < n) {
                const void* ff = memchr(d + e, 0xFF, n - 1 - e);
                if (!ff) { e = n - 1; break; }
                e = (size_t)((const uint8_t*)ff - d);
                const uint8_t nx = d[e + 1];
                if (nx != 0x00 && !(nx >= 0xD0 && nx <= 0xD7)) break;
                ++e;
            }
            j.scan_len = e - o;
            o = e;
            continue;
        }
        o += len;
    }
    if (!sof || !j.scan) return vd_set_error(VD_ERR_ARG, "jpeg: no frame / scan");
    j.hmax = j.vmax = 1;
    for (int i = 0; i < j.nc; ++i) {
        j.hmax = std::max(j.hmax, j.c[i].hs);
        j.vmax = std::max(j.vmax, j.c[i].vs);
    }
    if (j.nc == 1) j.c[0].hs = j.c[0].vs = j.hmax = j.vmax = 1;   // single component: one block per MCU
    j.mcux = (j.w + 8 * j.hmax - 1) / (8 * j.hmax);
    j.mcuy = (j.h + 8 * j.vmax - 1) / (8 * j.vmax);
    for (int i = 0; i < j.nc; ++i) {
        Comp& c = j.c[i];
        c.bw = j.mcux * c.hs;
        c.bh = j.mcuy * c.vs;
        if (!c.scanned) return vd_set_error(VD_ERR_ARG, "jpeg: component %d is not in the scan", i);
        if (!j.qpresent[c.tq] || !j.dc[c.td].present || !j.ac[c.ta].present)
            return vd_set_error(VD_ERR_ARG, "jpeg: component %d references a missing table", i);
    }
    return VD_OK;
}

// Bit reader over the entropy-coded segment: 0xFF00 -> 0xFF, a marker feeds zeros.
struct Bits {
    const uint8_t* d;
    size_t n, p = 0;
    uint64_t acc = 0;
    int nb = 0;
    bool marker = false;
    void fill() {
        // fast path: 4 bytes at once while none of them is 0xFF (no stuffing, no marker)
        while (nb <= 32 && !marker && p + 4 <= n) {
            uint32_t w;
            memcpy(&w, d + p, 4);
            if (((~w) - 0x01010101u) & w & 0x80808080u) break;   // a 0xFF byte among them (~w has a zero byte)
            w = __builtin_bswap32(w);
            acc |= (uint64_t)w << (32 - nb);
            nb += 32;
            p += 4;
        }
        while (nb <= 56) {
            uint32_t v = 0;
            if (!marker && p < n) {
                v = d[p];
                if (v == 0xFF) {
                    const uint32_t nx = p + 1 < n ? d[p + 1] : 0;
                    if (nx == 0x00) p += 2;
                    else { marker = true; v = 0; }
                } else {
                    ++p;
                }
            }
            acc |= (uint64_t)v << (56 - nb);
            nb += 8;
        }
    }
    inline uint32_t peek(int k) { if (nb < k) fill(); return (uint32_t)(acc >> (64 - k)); }
    inline void skip(int k) { acc <<= k; nb -= k; }
    inline int get(int k) {
        if (k == 0) return 0;
        const uint32_t v = peek(k);
        skip(k);
        return (int)v;
    }
    void restart() {   // discard buffered bits, step over the RSTn marker
        acc = 0;
        nb = 0;
        while (p + 1 < n && !(d[p] == 0xFF && d[p + 1] >= 0xD0 && d[p + 1] <= 0xD7)) ++p;
        if (p + 1 < n) p += 2;
        marker = false;
    }
};

inline int decode_sym(Bits& b, const Huff& h) {
    const uint32_t look = b.peek(kLook);
    const int l = h.look_len[look];
    if (l) {
        b.skip(l);
        return h.look_sym[look];
    }
    uint32_t code = b.peek(16);
    for (int len = 10; len <= 16; ++len) {
        const int c = (int)(code >> (16 - len));
        if (h.maxcode[len] >= 0 && c <= h.maxcode[len]) {
            b.skip(len);
            return h.vals[h.valoff[len] + c];
        }
    }
    return -1;
}

inline int extend(int v, int s) { return (s && v < (1 << (s - 1))) ? v - (1 << s) + 1 : v; }

// Entropy decode one image: entries (coefficient index << 16 | value) in MCU order
// into `ent` (at most 64 per block, written through a raw cursor into an
// uninitialised buffer), and per block, in block order (component, block row,
// block col), where[2 b] = its first entry, where[2 b + 1] = its entry count.
struct Entries {
    std::unique_ptr<uint32_t[]> ent;
    size_t n = 0;
    std::vector<uint32_t> where;
};

int entropy(const Info& j, Entries& out) {
    size_t nblk = 0;
    size_t cbase[3];
    for (int i = 0; i < j.nc; ++i) { cbase[i] = nblk; nblk += (size_t)j.c[i].bw * j.c[i].bh; }
    out.ent.reset(new uint32_t[nblk * 64 + 64]);
    uint32_t* const ent0 = out.ent.get();
    uint32_t* wp = ent0;
    std::vector<uint32_t>& where = out.where;
    where.assign(nblk * 2, 0u);
    Bits b{j.scan, j.scan_len};
    int pred[3] = {0, 0, 0};
    int mcu_n = 0;
    for (int my = 0; my < j.mcuy; ++my)
        for (int mx = 0; mx < j.mcux; ++mx) {
            if (j.restart && mcu_n && mcu_n % j.restart == 0) {
                b.restart();
                pred[0] = pred[1] = pred[2] = 0;
            }
            ++mcu_n;
            for (int ci = 0; ci < j.nc; ++ci) {
                const Comp& c = j.c[ci];
                const Huff& dc = j.dc[c.td];
                const Huff& ac = j.ac[c.ta];
                for (int by = 0; by < c.vs; ++by)
                    for (int bx = 0; bx < c.hs; ++bx) {
                        const size_t blk = cbase[ci] + (size_t)(my * c.vs + by) * c.bw + (mx * c.hs + bx);
                        where[2 * blk] = (uint32_t)(wp - ent0);
                        const int s = decode_sym(b, dc);
                        if (s < 0 || s > 11) return vd_set_error(VD_ERR_ARG, "jpeg: bad DC code");
                        pred[ci] += extend(b.get(s), s);
                        if (pred[ci]) *wp++ = (uint32_t)(0u << 16) | (uint16_t)(int16_t)pred[ci];
                        for (int k = 1; k < 64;) {
                            const uint32_t look = b.peek(kLook);
                            if (const int fl = ac.fa_len[look]) {   // code + extra bits in one look
                                b.skip(fl);
                                const int run = ac.fa_run[look];
                                if (run == 64) break;              // EOB
                                if (run == 16) { k += 16; continue; }   // ZRL
                                k += run;
                                if (k > 63) return vd_set_error(VD_ERR_ARG, "jpeg: AC run past the block");
                                *wp++ = ((uint32_t)kZigzag[k] << 16) | (uint16_t)ac.fa_val[look];
                                ++k;
                                continue;
                            }
                            const int rs = decode_sym(b, ac);
                            if (rs < 0) return vd_set_error(VD_ERR_ARG, "jpeg: bad AC code");
                            const int r = rs >> 4, sz = rs & 15;
                            if (sz == 0) {
                                if (r != 15) break;
                                k += 16;
                                continue;
                            }
                            k += r;
                            if (k > 63) return vd_set_error(VD_ERR_ARG, "jpeg: AC run past the block");
                            const int v = extend(b.get(sz), sz);
                            *wp++ = ((uint32_t)kZigzag[k] << 16) | (uint16_t)(int16_t)v;
                            ++k;
                        }
                        where[2 * blk + 1] = (uint32_t)(wp - ent0) - where[2 * blk];
                    }
            }
        }
    out.n = (size_t)(wp - ent0);
    return VD_OK;
}

bool same_layout(const Info& a, const Info& b) {
    if (a.h != b.h || a.w != b.w || a.nc != b.nc) return false;
    for (int i = 0; i < a.nc; ++i)
        if (a.c[i].hs != b.c[i].hs || a.c[i].vs != b.c[i].vs) return false;
    return true;
}

// ---- device entropy decode (jpeg_dec.hip) ------------------------------------
// Host part: table sets (deduplicated over the batch), scan segments copied 16-B
// aligned into one pinned buffer with the metadata, one H2D, then prep -> sync
// passes (until no chunk's exit state changes) -> scan -> write. Returns with
// *used = false (and nothing launched that matters) when the batch is not eligible
// (restart markers, table ids > 1, > 6 blocks per MCU) or the device flags a
// corrupt stream / no convergence: the caller then runs the host entropy stage,
// whose results and error messages are the reference behaviour.
void fill_tables(const Info& j, JLds& t) {
    memset(&t, 0, sizeof t);
    const Huff* hs[4] = {&j.dc[0], &j.dc[1], &j.ac[0], &j.ac[1]};
    for (int q = 0; q < 4; ++q) {
        const Huff& h = *hs[q];
        if (!h.present) continue;
        for (int i = 0; i < (1 << kLook); ++i) t.look[q][i] = (uint16_t)((h.look_len[i] << 8) | h.look_sym[i]);
        if (q >= 2)
            for (int i = 0; i < (1 << kLook); ++i)
                t.fast[q - 2][i] = (uint32_t)h.fa_len[i] | ((uint32_t)h.fa_run[i] << 8) | ((uint32_t)(uint16_t)h.fa_val[i] << 16);
        else   // DC: code + size bits within the lookahead, baseline sizes (<= 11) only
            for (int i = 0; i < (1 << kLook); ++i) {
                const int l = h.look_len[i], sz = h.look_sym[i];
                if (l == 0 || sz > 11 || l + sz > kLook) continue;
                const int extra = sz ? (i >> (kLook - l - sz)) & ((1 << sz) - 1) : 0;
                const int v = sz && extra < (1 << (sz - 1)) ? extra - (1 << sz) + 1 : extra;
                t.fastdc[q][i] = (uint32_t)(l + sz) | ((uint32_t)(uint16_t)v << 16);
            }
        for (int l = 0; l < 18; ++l) t.maxcode[q][l] = h.maxcode[l];
        for (int l = 0; l < 17; ++l) t.valoff[q][l] = h.valoff[l];
        memcpy(t.vals[q], h.vals, 256);
    }
}

int device_entropy(Ctx* ctx, const std::vector<Info>& info, int n, JpegArgs& a, size_t nblk_img, int nthreads,
                   bool* used) {
    *used = false;
    const Info& j0 = info[0];
    if (!ctx->tune.jdec_gpu) return VD_OK;
    int bpm = 0;
    for (int c = 0; c < j0.nc; ++c) bpm += j0.c[c].hs * j0.c[c].vs;
    if (bpm > 6) return VD_OK;
    for (int f = 0; f < n; ++f) {
        if (info[f].restart) return VD_OK;
        for (int c = 0; c < j0.nc; ++c)
            if (info[f].c[c].td > 1 || info[f].c[c].ta > 1 || !info[f].dc[info[f].c[c].td].present ||
                !info[f].ac[info[f].c[c].ta].present)
                return VD_OK;
        if (info[f].scan_len >= (1u << 28)) return VD_OK;
    }
    JdecLaunch L{};
    L.n = n; L.bpm = bpm;
    {
        int u = 0;
        for (int c = 0; c < j0.nc; ++c)
            for (int by = 0; by < j0.c[c].vs; ++by)
                for (int bx = 0; bx < j0.c[c].hs; ++bx, ++u) {
                    L.ucomp[u] = c; L.udc[u] = j0.c[c].td; L.uac[u] = j0.c[c].ta; L.ubx[u] = bx; L.uby[u] = by;
                }
    }
    L.mcux = j0.mcux;
    L.total_blocks = j0.mcux * j0.mcuy * bpm;
    for (int c = 0; c < 3; ++c) { L.cblk[c] = a.cblk[c]; L.bw[c] = a.bw[c]; L.hs[c] = a.hs[c]; L.vs[c] = a.vs[c]; }
    L.blocks_per_image = (int)nblk_img;
    // per-frame table sets (the component -> table ids are the batch's: same layout)
    for (int f = 1; f < n; ++f)
        for (int c = 0; c < j0.nc; ++c)
            if (info[f].c[c].td != j0.c[c].td || info[f].c[c].ta != j0.c[c].ta) return VD_OK;
    std::vector<JLds> sets;
    std::vector<uint8_t> tab_of(n);
    JLds tmp;
    for (int f = 0; f < n; ++f) {
        fill_tables(info[f], tmp);
        size_t k = 0;
        while (k < sets.size() && memcmp(&sets[k], &tmp, sizeof tmp)) ++k;
        if (k == sets.size()) {
            if (sets.size() >= 255) return VD_OK;
            sets.push_back(tmp);
        }
        tab_of[f] = (uint8_t)k;
    }
    const int C = std::max(16, ctx->tune.jdec_chunk / 16 * 16);
    L.chunk_bytes = C;
    std::vector<uint32_t> seg_off(n), seg_len(n), chunk0(n + 1);
    std::vector<int> wg_frame;
    std::vector<uint32_t> wg_chunk;
    size_t bytes_total = 0;
    uint32_t nc_total = 0;
    for (int f = 0; f < n; ++f) {
        seg_off[f] = (uint32_t)bytes_total;
        seg_len[f] = (uint32_t)info[f].scan_len;
        bytes_total += (info[f].scan_len + 80 + 15) / 16 * 16;             // 64-B reader buffers read past the end
        chunk0[f] = nc_total;
        const uint32_t nch = std::max<uint32_t>(1, (uint32_t)((info[f].scan_len + C - 1) / C));
        for (uint32_t c = 0; c < nch; c += 256) { wg_frame.push_back(f); wg_chunk.push_back(c); }
        nc_total += nch;
    }
    chunk0[n] = nc_total;
    if (bytes_total >= (1ull << 32)) return VD_OK;
    const int nwg = (int)wg_frame.size();
    // pinned image: metadata | quant | tables | segments
    auto al = [](size_t x) { return (x + 255) / 256 * 256; };
    const size_t o_soff = 0, o_slen = al(o_soff + n * 4), o_c0 = al(o_slen + n * 4), o_tab = al(o_c0 + (n + 1) * 4);
    const size_t o_wgf = al(o_tab + n), o_wgc = al(o_wgf + nwg * 4), o_q = al(o_wgc + nwg * 4);
    const size_t o_tabs = al(o_q + (size_t)n * 3 * 64 * 2), o_bytes = al(o_tabs + sets.size() * sizeof(JLds));
    const size_t himg = o_bytes + bytes_total;
    int rc;
    VD_CHECK_HIP(hipEventSynchronize(ctx->jpeg_ev));                     // the previous H2D from it is done
    if ((rc = ctx->ensure_pinned(&ctx->jdec_host, &ctx->jdec_host_bytes, himg))) return rc;
    if ((rc = ctx->ensure_staging(&ctx->jdec_dev, &ctx->jdec_dev_bytes, himg))) return rc;
    char* hp = (char*)ctx->jdec_host;
    memcpy(hp + o_soff, seg_off.data(), n * 4);
    memcpy(hp + o_slen, seg_len.data(), n * 4);
    memcpy(hp + o_c0, chunk0.data(), (n + 1) * 4);
    memcpy(hp + o_tab, tab_of.data(), n);
    memcpy(hp + o_wgf, wg_frame.data(), nwg * 4);
    memcpy(hp + o_wgc, wg_chunk.data(), nwg * 4);
    memcpy(hp + o_tabs, sets.data(), sets.size() * sizeof(JLds));
    uint16_t* hq = (uint16_t*)(hp + o_q);
    std::atomic<int> next{0};
    auto copier = [&]() {
        for (int f; (f = next.fetch_add(1)) < n;) {
            char* dst = hp + o_bytes + seg_off[f];
            memcpy(dst, info[f].scan, info[f].scan_len);
            memset(dst + info[f].scan_len, 0, (info[f].scan_len + 95) / 16 * 16 - info[f].scan_len);
            for (int c = 0; c < j0.nc; ++c) memcpy(hq + ((size_t)f * 3 + c) * 64, info[f].q[info[f].c[c].tq], 128);
        }
    };
    {
        std::vector<std::thread> pool;
        for (int t = 1; t < nthreads; ++t) pool.emplace_back(copier);
        copier();
        for (auto& t : pool) t.join();
    }
    VD_CHECK_HIP(hipMemcpyAsync(ctx->jdec_dev, hp, himg, hipMemcpyHostToDevice, ctx->stream));
    VD_CHECK_HIP(hipEventRecord(ctx->jpeg_ev, ctx->stream));
    // device work area: per chunk state + the dense blocks
    const size_t NC = nc_total;
    const int R = std::min(255, std::max(0, ctx->tune.jdec_sync));
    const size_t w_D = 0, w_S = al(w_D + (NC + n) * 4), w_Su = al(w_S + NC * 4), w_E0 = al(w_Su + NC);
    const size_t w_E1 = al(w_E0 + NC * 4), w_U0 = al(w_E1 + NC * 4), w_U1 = al(w_U0 + NC), w_nb = al(w_U1 + NC);
    const size_t w_dcs = al(w_nb + NC * 4), w_base = al(w_dcs + NC * 12), w_dco = al(w_base + NC * 4);
    const size_t w_fl = al(w_dco + NC * 12), w_own = al(w_fl + 4 * (4 + 65)), w_sel = al(w_own + NC * 4);
    size_t w_L[2][4], o = al(w_sel + NC);
    for (int k = 0; k < 2; ++k) {   // Lpos, Lu, Ldc, Lcnt
        w_L[k][0] = o; w_L[k][1] = al(o + NC * R * 4); w_L[k][2] = al(w_L[k][1] + NC * R);
        w_L[k][3] = al(w_L[k][2] + NC * R * 12); o = al(w_L[k][3] + NC);
    }
    const size_t w_dense = o;
    const size_t wbytes = w_dense + (size_t)n * nblk_img * 128;
    if ((rc = ctx->ensure_staging(&ctx->jdec_work, &ctx->jdec_work_bytes, wbytes))) return rc;
    char* dp = (char*)ctx->jdec_dev;
    char* wp = (char*)ctx->jdec_work;
    L.seg_off = (const uint32_t*)(dp + o_soff); L.seg_len = (const uint32_t*)(dp + o_slen);
    L.chunk0 = (const uint32_t*)(dp + o_c0); L.tab_of = (const uint8_t*)(dp + o_tab);
    L.wg_frame = (const int*)(dp + o_wgf); L.wg_chunk = (const uint32_t*)(dp + o_wgc);
    L.tabs = (const JLds*)(dp + o_tabs); L.bytes = (const uint8_t*)(dp + o_bytes);
    L.D = (uint32_t*)(wp + w_D); L.S = (uint32_t*)(wp + w_S); L.Su = (uint8_t*)(wp + w_Su);
    L.Epos[0] = (uint32_t*)(wp + w_E0); L.Epos[1] = (uint32_t*)(wp + w_E1);
    L.Eu[0] = (uint8_t*)(wp + w_U0); L.Eu[1] = (uint8_t*)(wp + w_U1);
    L.nblk = (uint32_t*)(wp + w_nb); L.dcs = (int*)(wp + w_dcs); L.base = (uint32_t*)(wp + w_base);
    L.dcoff = (int*)(wp + w_dco); L.flags = (int*)(wp + w_fl); L.dense = (int16_t*)(wp + w_dense);
    L.own = (uint32_t*)(wp + w_own); L.Lsel = (uint8_t*)(wp + w_sel); L.R = R;
    for (int k = 0; k < 2; ++k) {
        L.Lpos[k] = (uint32_t*)(wp + w_L[k][0]); L.Lu[k] = (uint8_t*)(wp + w_L[k][1]);
        L.Ldc[k] = (int*)(wp + w_L[k][2]); L.Lcnt[k] = (uint8_t*)(wp + w_L[k][3]);
    }
    L.nwg = nwg;
    hipError_t e;
    auto launch = [&](int stage, const char* what) -> int {
        L.stage = stage;
        if ((e = vd_launch_jdec(L, ctx->stream)) != hipSuccess) return vd_set_error(VD_ERR_HIP, "jdec %s: %s", what, hipGetErrorString(e));
        return VD_OK;
    };
    if ((rc = launch(0, "prep"))) return rc;
    VD_CHECK_HIP(hipMemsetAsync(L.flags, 0, 4 * (4 + 65), ctx->stream));
    L.pass = 0;
    if ((rc = launch(1, "pass"))) return rc;
    // resynchronisation passes in groups of jdec_group between host checks (a pass after
    // convergence only copies exit states), until one changes no exit state
    const int grp = std::max(1, ctx->tune.jdec_group);
    int pf[65] = {0};
    int pass = 1, conv = 0;
    while (!conv && pass <= 64) {
        const int last = std::min(64, pass + grp - 1);
        for (int p = pass; p <= last; ++p) {
            L.pass = p;
            if ((rc = launch(1, "pass"))) return rc;
        }
        VD_CHECK_HIP(hipMemcpyAsync(pf + pass, L.flags + 4 + pass, 4 * (last - pass + 1), hipMemcpyDeviceToHost, ctx->stream));
        VD_CHECK_HIP(hipStreamSynchronize(ctx->stream));
        for (int p = pass; p <= last && !conv; ++p)
            if (pf[p] == 0) conv = p;
        pass = last + 1;
    }
    ctx->jdec_passes = conv ? conv + 1 : 65;
    if (!conv) return VD_OK;                                          // no convergence: host decode
    int flag[4] = {0, 0, 0, 0};
    // the write stores each coefficient straight into its dense block: zeros first
    VD_CHECK_HIP(hipMemsetAsync(L.dense, 0, (size_t)n * nblk_img * 128, ctx->stream));
    if ((rc = launch(2, "scan")) || (rc = launch(3, "write"))) return rc;
    VD_CHECK_HIP(hipMemcpyAsync(flag, L.flags, 8, hipMemcpyDeviceToHost, ctx->stream));
    VD_CHECK_HIP(hipStreamSynchronize(ctx->stream));
    if (flag[1] != 0) return VD_OK;                                    // corrupt: the host decoder reports it
    a.dense = L.dense;
    a.quant = (const uint16_t*)(dp + o_q);
    a.blk_off = nullptr;
    a.entries = nullptr;
    *used = true;
    return VD_OK;
}

}  // namespace

extern "C" int vd_jpeg_info(const uint8_t* data, size_t size, int* h, int* w, int* comps) {
    if (!data) return vd_set_error(VD_ERR_ARG, "null data");
    Info j;
    int rc = parse(data, size, j, true);
    if (rc) return rc;
    if (h) *h = j.h;
    if (w) *w = j.w;
    if (comps) *comps = j.nc;
    return VD_OK;
}

// Test hook: the host entropy stage alone (no GPU): quantized coefficients of every
// block, natural order, block order (component, block row, block col).
extern "C" int vdt_jpeg_coefficients(const uint8_t* data, size_t size, int16_t* out, size_t cap_blocks,
                                     int* nblocks) {
    if (!data) return vd_set_error(VD_ERR_ARG, "null data");
    Info j;
    Entries en;
    int rc = parse(data, size, j);
    if (!rc) rc = entropy(j, en);
    if (rc) return rc;
    const size_t nb = en.where.size() / 2;
    if (nblocks) *nblocks = (int)nb;
    if (!out) return VD_OK;
    if (cap_blocks < nb) return vd_set_error(VD_ERR_ARG, "need %zu blocks", nb);
    memset(out, 0, nb * 64 * 2);
    for (size_t b = 0; b < nb; ++b)
        for (uint32_t e = 0; e < en.where[2 * b + 1]; ++e) {
            const uint32_t v = en.ent[en.where[2 * b] + e];
            out[b * 64 + (v >> 16)] = (int16_t)(v & 0xFFFF);
        }
    return VD_OK;
}

extern "C" int vdt_jdec_stats(vd_ctx* hctx, int* passes) {
    Ctx* ctx = (Ctx*)hctx;
    if (!ctx) return vd_set_error(VD_ERR_ARG, "null context");
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (passes) *passes = ctx->jdec_passes;
    return VD_OK;
}

static int launch_idct_color(Ctx* ctx, JpegArgs& a, uint8_t* out, int fh, size_t pitch, int where, int n);

extern "C" int vd_jpeg_decode(vd_ctx* hctx, const uint8_t* const* data, const size_t* sizes, int n, uint8_t* out,
                              int fh, int fw, size_t pitch, int where) {
    Ctx* ctx = (Ctx*)hctx;
    if (!ctx) return vd_set_error(VD_ERR_ARG, "null context");
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (hipSetDevice(ctx->device) != hipSuccess) return vd_set_error(VD_ERR_HIP, "hipSetDevice(%d) failed", ctx->device);
    if (!data || !sizes || !out || n <= 0 || n > ctx->cfg.max_batch || fh <= 0 || fw <= 0 || pitch < (size_t)fw * 3)
        return vd_set_error(VD_ERR_ARG, "vd_jpeg_decode: bad arguments");
    // 1) parse every frame's headers (and find its entropy-coded segment), host threads
    std::vector<Info> info(n);
    std::vector<Entries> ent(n);
    std::vector<int> rcs(n, VD_OK);
    std::vector<std::string> errs(n);
    std::atomic<int> next{0};
    const int nthreads = std::max(1, std::min(n, ctx->jpeg_threads));
    auto run_threads = [&](auto&& fn) {
        next = 0;
        std::vector<std::thread> pool;
        for (int t = 1; t < nthreads; ++t) pool.emplace_back(fn);
        fn();
        for (auto& t : pool) t.join();
    };
    run_threads([&]() {
        for (int i; (i = next.fetch_add(1)) < n;) {
            int rc = parse(data[i], sizes[i], info[i]);
            if (!rc && (info[i].h != fh || info[i].w != fw))
                rc = vd_set_error(VD_ERR_ARG, "jpeg %d is %dx%d, expected %dx%d", i, info[i].w, info[i].h, fw, fh);
            rcs[i] = rc;
            if (rc) errs[i] = vd_last_error();
        }
    });
    for (int i = 0; i < n; ++i)
        if (rcs[i]) return vd_set_error(rcs[i], "jpeg %d: %s", i, errs[i].c_str());
    for (int i = 1; i < n; ++i)
        if (!same_layout(info[0], info[i]))
            return vd_set_error(VD_ERR_ARG, "jpeg %d: component layout differs from jpeg 0 (one call decodes one stream)", i);
    const Info& j0 = info[0];
    JpegArgs a{};
    a.n = n; a.h = fh; a.w = fw; a.nc = j0.nc; a.hmax = j0.hmax; a.vmax = j0.vmax;
    size_t nblk_img = 0;
    for (int c = 0; c < j0.nc; ++c) {
        a.bw[c] = j0.c[c].bw; a.bh[c] = j0.c[c].bh; a.hs[c] = j0.c[c].hs; a.vs[c] = j0.c[c].vs;
        a.cblk[c] = (int)nblk_img;
        a.plane_off[c] = (long)nblk_img * 64;          // plane bytes = blocks * 64, same order
        nblk_img += (size_t)a.bw[c] * a.bh[c];
    }
    a.blocks_per_image = (int)nblk_img;
    int rc;
    // 2a) entropy decode on the device (jpeg_dec.hip) when the batch allows it
    bool dev_done = false;
    if ((rc = device_entropy(ctx, info, n, a, nblk_img, nthreads, &dev_done))) return rc;
    if (dev_done) {
        if ((rc = ctx->ensure_staging(&ctx->jpeg_planes, &ctx->jpeg_planes_bytes, nblk_img * n * 64 + 64))) return rc;
        a.planes = (uint8_t*)ctx->jpeg_planes;
        return launch_idct_color(ctx, a, out, fh, pitch, where, n);
    }
    // 2b) entropy decode on host threads into sparse coefficient lists
    run_threads([&]() {
        for (int i; (i = next.fetch_add(1)) < n;) {
            const int rc = entropy(info[i], ent[i]);
            rcs[i] = rc;
            if (rc) errs[i] = vd_last_error();
        }
    });
    for (int i = 0; i < n; ++i)
        if (rcs[i]) return vd_set_error(rcs[i], "jpeg %d: %s", i, errs[i].c_str());
    // pack: per image [blocks] offsets (global), entries, quant tables
    size_t tot_ent = 0;
    for (int i = 0; i < n; ++i) tot_ent += ent[i].n;
    const size_t nblk = nblk_img * n;
    const size_t off_bytes = (nblk + 1) * 4, q_bytes = (size_t)n * 3 * 64 * 2, ent_bytes = std::max<size_t>(tot_ent, 1) * 4;
    const size_t need = off_bytes + q_bytes + ent_bytes + 64;
    if ((rc = ctx->ensure_pinned(&ctx->jpeg_host, &ctx->jpeg_host_bytes, need))) return rc;
    if ((rc = ctx->ensure_staging(&ctx->jpeg_dev, &ctx->jpeg_dev_bytes, need))) return rc;
    const size_t plane_bytes = nblk * 64;
    if ((rc = ctx->ensure_staging(&ctx->jpeg_planes, &ctx->jpeg_planes_bytes, plane_bytes + 64))) return rc;
    // the previous call's H2D from the pinned buffer must be done before it is rewritten
    VD_CHECK_HIP(hipEventSynchronize(ctx->jpeg_ev));
    char* hp = (char*)ctx->jpeg_host;
    uint32_t* hoff = (uint32_t*)hp;
    uint16_t* hq = (uint16_t*)(hp + off_bytes);
    uint32_t* hent = (uint32_t*)(hp + off_bytes + q_bytes);
    // per-image entry bases, then the packing itself on the same host threads (a
    // noise 1080p frame carries ~11 MB of entries: a serial copy would rival the decode)
    std::vector<size_t> ebase(n + 1, 0);
    for (int i = 0; i < n; ++i) ebase[i + 1] = ebase[i] + ent[i].n;
    next = 0;
    std::vector<std::thread> pool;
    auto packer = [&]() {
        for (int i; (i = next.fetch_add(1)) < n;) {
            // regroup MCU order -> block order straight into the pinned buffer
            size_t o = ebase[i], b = (size_t)i * nblk_img;
            const std::vector<uint32_t>& wh = ent[i].where;
            for (size_t k = 0; k < nblk_img; ++k, ++b) {
                const uint32_t st = wh[2 * k], cn = wh[2 * k + 1];
                hoff[b] = (uint32_t)o;
                memcpy(hent + o, ent[i].ent.get() + st, (size_t)cn * 4);
                o += cn;
            }
            for (int c = 0; c < j0.nc; ++c) memcpy(hq + ((size_t)i * 3 + c) * 64, info[i].q[info[i].c[c].tq], 128);
        }
    };
    pool.clear();
    for (int t = 1; t < nthreads; ++t) pool.emplace_back(packer);
    packer();
    for (auto& t : pool) t.join();
    hoff[nblk] = (uint32_t)ebase[n];
    VD_CHECK_HIP(hipMemcpyAsync(ctx->jpeg_dev, ctx->jpeg_host, off_bytes + q_bytes + tot_ent * 4,
                                hipMemcpyHostToDevice, ctx->stream));
    VD_CHECK_HIP(hipEventRecord(ctx->jpeg_ev, ctx->stream));
    char* dp = (char*)ctx->jpeg_dev;
    a.blk_off = (const uint32_t*)dp;
    a.quant = (const uint16_t*)(dp + off_bytes);
    a.entries = (const uint32_t*)(dp + off_bytes + q_bytes);
    a.planes = (uint8_t*)ctx->jpeg_planes;
    return launch_idct_color(ctx, a, out, fh, pitch, where, n);
}

// 3) device: IDCT into planes, then upsample + color into the frames
static int launch_idct_color(Ctx* ctx, JpegArgs& a, uint8_t* out, int fh, size_t pitch, int where, int n) {
    int rc;
    uint8_t* dout = out;
    if (where == VD_HOST) {
        if ((rc = ctx->ensure_staging(&ctx->stage_in, &ctx->stage_in_bytes, (size_t)n * fh * pitch))) return rc;
        dout = (uint8_t*)ctx->stage_in;
    }
    a.out = dout; a.pitch = pitch;
    ctx->t_begin(4, 0);
    hipError_t e = vd_launch_jpeg(a, ctx->stream);
    ctx->t_end();
    if (e != hipSuccess) return vd_set_error(VD_ERR_HIP, "jpeg kernels: %s", hipGetErrorString(e));
    if (where == VD_HOST) {
        VD_CHECK_HIP(hipMemcpyAsync(out, dout, (size_t)n * fh * pitch, hipMemcpyDeviceToHost, ctx->stream));
        VD_CHECK_HIP(hipStreamSynchronize(ctx->stream));
    }
    return VD_OK;
}
