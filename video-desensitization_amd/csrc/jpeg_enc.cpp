// jpeg_enc.cpp — host stage of the JPEG frame encode: vd_jpeg_encode.
//
// Replaces the frame write of the reference's loop, cv2.imwrite of every
// processed frame (combine_detect.py:174-180, :259-262; create_video reads them
// back, :479-595), with libjpeg-turbo's default compressor restated bit-exactly
// (oracle/jpeg_enc.py; quality 95 and 4:2:0 are cv2's defaults):
//   1. device (jpeg_enc.hip): colour conversion, downsampling, edge replication,
//      ISLOW FDCT and reciprocal quantisation of every block of the batch;
//   2. one D2H of the int16 coefficient blocks into pinned memory;
//   3. host threads, one frame each: the jchuff.c sequential Huffman stage in MCU
//      order (standard Annex K tables, dummy blocks at the right / bottom MCU edge
//      with their neighbour's DC as jccoefct.c makes them, 0xFF stuffing, 1-bit
//      padding) behind the JFIF / DQT / SOF0 / DHT / SOS headers libjpeg writes.
#include "../../include/vdmi.h"
#include "vd_common.h"
#include "nets.h"

#include <algorithm>
#include <atomic>
#include <cstring>
#include <thread>
#include <vector>

namespace {

const uint8_t kZigzag[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48,
                             41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23,
                             30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};
const uint8_t kStdLuma[64] = {16, 11, 10, 16, 24,  40,  51,  61,  12, 12, 14, 19, 26,  58,  60,  55,
                              14, 13, 16, 24, 40,  57,  69,  56,  14, 17, 22, 29, 51,  87,  80,  62,
                              18, 22, 37, 56, 68,  109, 103, 77,  24, 35, 55, 64, 81,  104, 113, 92,
                              49, 64, 78, 87, 103, 121, 120, 101, 72, 92, 95, 98, 112, 100, 103, 99};
const uint8_t kStdChroma[64] = {17, 18, 24, 47, 99, 99, 99, 99, 18, 21, 26, 66, 99, 99, 99, 99, 24, 26, 56, 99, 99, 99,
                                99, 99, 47, 66, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99,
                                99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99};
// Annex K.3: bits[1..16] then values
const uint8_t kDcLumaBits[16] = {0, 1, 5, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0};
const uint8_t kDcChromaBits[16] = {0, 3, 1, 1, 1, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0};
const uint8_t kDcVals[12] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11};
const uint8_t kAcLumaBits[16] = {0, 2, 1, 3, 3, 2, 4, 3, 5, 5, 4, 4, 0, 0, 1, 0x7d};
const uint8_t kAcLumaVals[162] = {
    0x01, 0x02, 0x03, 0x00, 0x04, 0x11, 0x05, 0x12, 0x21, 0x31, 0x41, 0x06, 0x13, 0x51, 0x61, 0x07, 0x22, 0x71, 0x14,
    0x32, 0x81, 0x91, 0xa1, 0x08, 0x23, 0x42, 0xb1, 0xc1, 0x15, 0x52, 0xd1, 0xf0, 0x24, 0x33, 0x62, 0x72, 0x82, 0x09,
    0x0a, 0x16, 0x17, 0x18, 0x19, 0x1a, 0x25, 0x26, 0x27, 0x28, 0x29, 0x2a, 0x34, 0x35, 0x36, 0x37, 0x38, 0x39, 0x3a,
    0x43, 0x44, 0x45, 0x46, 0x47, 0x48, 0x49, 0x4a, 0x53, 0x54, 0x55, 0x56, 0x57, 0x58, 0x59, 0x5a, 0x63, 0x64, 0x65,
    0x66, 0x67, 0x68, 0x69, 0x6a, 0x73, 0x74, 0x75, 0x76, 0x77, 0x78, 0x79, 0x7a, 0x83, 0x84, 0x85, 0x86, 0x87, 0x88,
    0x89, 0x8a, 0x92, 0x93, 0x94, 0x95, 0x96, 0x97, 0x98, 0x99, 0x9a, 0xa2, 0xa3, 0xa4, 0xa5, 0xa6, 0xa7, 0xa8, 0xa9,
    0xaa, 0xb2, 0xb3, 0xb4, 0xb5, 0xb6, 0xb7, 0xb8, 0xb9, 0xba, 0xc2, 0xc3, 0xc4, 0xc5, 0xc6, 0xc7, 0xc8, 0xc9, 0xca,
    0xd2, 0xd3, 0xd4, 0xd5, 0xd6, 0xd7, 0xd8, 0xd9, 0xda, 0xe1, 0xe2, 0xe3, 0xe4, 0xe5, 0xe6, 0xe7, 0xe8, 0xe9, 0xea,
    0xf1, 0xf2, 0xf3, 0xf4, 0xf5, 0xf6, 0xf7, 0xf8, 0xf9, 0xfa};
const uint8_t kAcChromaBits[16] = {0, 2, 1, 2, 4, 4, 3, 4, 7, 5, 4, 4, 0, 1, 2, 0x77};
const uint8_t kAcChromaVals[162] = {
    0x00, 0x01, 0x02, 0x03, 0x11, 0x04, 0x05, 0x21, 0x31, 0x06, 0x12, 0x41, 0x51, 0x07, 0x61, 0x71, 0x13, 0x22, 0x32,
    0x81, 0x08, 0x14, 0x42, 0x91, 0xa1, 0xb1, 0xc1, 0x09, 0x23, 0x33, 0x52, 0xf0, 0x15, 0x62, 0x72, 0xd1, 0x0a, 0x16,
    0x24, 0x34, 0xe1, 0x25, 0xf1, 0x17, 0x18, 0x19, 0x1a, 0x26, 0x27, 0x28, 0x29, 0x2a, 0x35, 0x36, 0x37, 0x38, 0x39,
    0x3a, 0x43, 0x44, 0x45, 0x46, 0x47, 0x48, 0x49, 0x4a, 0x53, 0x54, 0x55, 0x56, 0x57, 0x58, 0x59, 0x5a, 0x63, 0x64,
    0x65, 0x66, 0x67, 0x68, 0x69, 0x6a, 0x73, 0x74, 0x75, 0x76, 0x77, 0x78, 0x79, 0x7a, 0x82, 0x83, 0x84, 0x85, 0x86,
    0x87, 0x88, 0x89, 0x8a, 0x92, 0x93, 0x94, 0x95, 0x96, 0x97, 0x98, 0x99, 0x9a, 0xa2, 0xa3, 0xa4, 0xa5, 0xa6, 0xa7,
    0xa8, 0xa9, 0xaa, 0xb2, 0xb3, 0xb4, 0xb5, 0xb6, 0xb7, 0xb8, 0xb9, 0xba, 0xc2, 0xc3, 0xc4, 0xc5, 0xc6, 0xc7, 0xc8,
    0xc9, 0xca, 0xd2, 0xd3, 0xd4, 0xd5, 0xd6, 0xd7, 0xd8, 0xd9, 0xda, 0xe2, 0xe3, 0xe4, 0xe5, 0xe6, 0xe7, 0xe8, 0xe9,
    0xea, 0xf2, 0xf3, 0xf4, 0xf5, 0xf6, 0xf7, 0xf8, 0xf9, 0xfa};

struct HuffEnc {   // jchuff.c jpeg_make_c_derived_tbl: code and size per symbol
    uint16_t code[256];
    uint8_t size[256];
    void build(const uint8_t* bits, const uint8_t* vals) {
        memset(size, 0, sizeof(size));
        unsigned c = 0;
        int k = 0;
        for (int l = 1; l <= 16; ++l) {
            for (int i = 0; i < bits[l - 1]; ++i, ++k) {
                code[vals[k]] = (uint16_t)c++;
                size[vals[k]] = (uint8_t)l;
            }
            c <<= 1;
        }
    }
};

struct Tables {
    HuffEnc dc[2], ac[2];
    Tables() {
        dc[0].build(kDcLumaBits, kDcVals);
        dc[1].build(kDcChromaBits, kDcVals);
        ac[0].build(kAcLumaBits, kAcLumaVals);
        ac[1].build(kAcChromaBits, kAcChromaVals);
    }
};
const Tables& tables() {
    static const Tables t;
    return t;
}

// jpeg_set_quality -> jpeg_quality_scaling + jpeg_add_quant_table(force_baseline = TRUE)
void quant_table(const uint8_t* std, int quality, uint16_t* q) {
    quality = std::max(1, std::min(100, quality));
    const int scale = quality < 50 ? 5000 / quality : 200 - 2 * quality;
    for (int i = 0; i < 64; ++i) q[i] = (uint16_t)std::max(1, std::min(255, (std[i] * scale + 50) / 100));
}

// compute_reciprocal (jcdctmgr.c), 16-bit DCTELEM of libjpeg-turbo's SIMD build
void reciprocal(int divisor, uint16_t* recip, uint16_t* corr, uint8_t* shift) {
    int b = 31 - __builtin_clz((unsigned)divisor);
    int r = 16 + b;
    unsigned fq = (1u << r) / divisor, fr = (1u << r) % divisor, c = divisor / 2;
    if (fr == 0) { fq >>= 1; --r; }
    else if (fr <= (unsigned)divisor / 2) ++c;
    else ++fq;
    *recip = (uint16_t)fq;
    *corr = (uint16_t)c;
    *shift = (uint8_t)r;
}

struct BitOut {   // jchuff.c emit_bits / flush_bits with 0xFF stuffing
    uint8_t* p;
    uint8_t* end;
    uint64_t acc = 0;   // the low n bits are pending, oldest first
    int n = 0;          // < 32 between calls
    bool overflow = false;
    inline void byte(uint8_t b) {
        *p++ = b;
        if (b == 0xFF) *p++ = 0;
    }
    inline void put(unsigned code, int size) {   // size <= 27
        acc = (acc << size) | (code & ((1u << size) - 1));
        n += size;
        if (n < 32) return;
        n -= 32;
        const uint32_t w = (uint32_t)(acc >> n);
        if (p + 8 > end) { overflow = true; p = end - 8; }
        const uint32_t x = ~w;                   // a 0xFF byte of w is a zero byte of x
        if (!((x - 0x01010101u) & ~x & 0x80808080u)) {   // common case: 4 bytes, no stuffing
            const uint32_t be = __builtin_bswap32(w);
            memcpy(p, &be, 4);
            p += 4;
        } else {
            byte((uint8_t)(w >> 24)); byte((uint8_t)(w >> 16)); byte((uint8_t)(w >> 8)); byte((uint8_t)w);
        }
    }
    void flush() {      // seven 1-bits fill the partial byte; whole bytes out, the rest dropped
        acc = (acc << 7) | 0x7F;
        n += 7;
        while (n >= 8) {
            n -= 8;
            if (p + 2 > end) { overflow = true; return; }
            byte((uint8_t)(acc >> n));
        }
        acc = 0;
        n = 0;
    }
};

inline int nbits(int v) { return v ? 32 - __builtin_clz((unsigned)(v < 0 ? -v : v)) : 0; }

// encode_one_block (jchuff.c); blk in natural order
inline void encode_block(BitOut& o, const int16_t* blk, int& last_dc, const HuffEnc& dc, const HuffEnc& ac) {
    int diff = blk[0] - last_dc;
    last_dc = blk[0];
    int nb = nbits(diff);
    // code and extra bits in one put (<= 16 + 11 bits)
    o.put(((unsigned)dc.code[nb] << nb) | ((unsigned)(diff < 0 ? diff - 1 : diff) & ((1u << nb) - 1)), dc.size[nb] + nb);
    int r = 0;
    for (int k = 1; k < 64; ++k) {
        const int v = blk[kZigzag[k]];
        if (v == 0) { ++r; continue; }
        while (r > 15) { o.put(ac.code[0xF0], ac.size[0xF0]); r -= 16; }
        nb = nbits(v);
        const int sym = (r << 4) + nb;
        o.put(((unsigned)ac.code[sym] << nb) | ((unsigned)(v < 0 ? v - 1 : v) & ((1u << nb) - 1)), ac.size[sym] + nb);
        r = 0;
    }
    if (r) o.put(ac.code[0], ac.size[0]);
}

void put16(uint8_t*& p, int v) { *p++ = (uint8_t)(v >> 8); *p++ = (uint8_t)v; }

void put_dht(uint8_t*& p, int tc, int th, const uint8_t* bits, const uint8_t* vals) {
    int nv = 0;
    for (int i = 0; i < 16; ++i) nv += bits[i];
    *p++ = 0xFF; *p++ = 0xC4;
    put16(p, 2 + 1 + 16 + nv);
    *p++ = (uint8_t)(tc << 4 | th);
    memcpy(p, bits, 16); p += 16;
    memcpy(p, vals, nv); p += nv;
}

struct Geo {
    int h, w, hl, vl;
    int bw[3], bh[3];
    long cblk[3], bpf;
};

// JFIF / DQT / SOF0 / DHT / SOS headers as libjpeg writes them; returns their length
size_t write_headers(const Geo& g, const uint16_t* ql, const uint16_t* qc, uint8_t* out) {
    uint8_t* p = out;
    static const uint8_t head[] = {0xFF, 0xD8, 0xFF, 0xE0, 0x00, 0x10, 'J', 'F', 'I', 'F', 0x00,
                                   0x01, 0x01, 0x00, 0x00, 0x01, 0x00, 0x01, 0x00, 0x00};
    memcpy(p, head, sizeof(head)); p += sizeof(head);
    for (int t = 0; t < 2; ++t) {
        const uint16_t* q = t ? qc : ql;
        *p++ = 0xFF; *p++ = 0xDB; put16(p, 67); *p++ = (uint8_t)t;
        for (int k = 0; k < 64; ++k) *p++ = (uint8_t)q[kZigzag[k]];
    }
    *p++ = 0xFF; *p++ = 0xC0; put16(p, 17); *p++ = 8; put16(p, g.h); put16(p, g.w); *p++ = 3;
    const uint8_t sof[9] = {1, (uint8_t)(g.hl << 4 | g.vl), 0, 2, 0x11, 1, 3, 0x11, 1};
    memcpy(p, sof, 9); p += 9;
    put_dht(p, 0, 0, kDcLumaBits, kDcVals);
    put_dht(p, 1, 0, kAcLumaBits, kAcLumaVals);
    put_dht(p, 0, 1, kDcChromaBits, kDcVals);
    put_dht(p, 1, 1, kAcChromaBits, kAcChromaVals);
    static const uint8_t sos[] = {0xFF, 0xDA, 0x00, 0x0C, 0x03, 0x01, 0x00, 0x02, 0x11, 0x03, 0x11, 0x00, 0x3F, 0x00};
    memcpy(p, sos, sizeof(sos)); p += sizeof(sos);
    return (size_t)(p - out);
}

// one frame: headers + entropy-coded segment + EOI; returns bytes or 0 on overflow
size_t encode_frame(const Geo& g, const int16_t* coef, const uint16_t* ql, const uint16_t* qc, uint8_t* out,
                    size_t cap) {
    if (cap < 1024) return 0;
    uint8_t* p = out + write_headers(g, ql, qc, out);
    const Tables& T = tables();
    BitOut o{p, out + cap - 2};
    int last[3] = {0, 0, 0};
    int16_t dummy[64];
    const int mcux = (g.w + 8 * g.hl - 1) / (8 * g.hl), mcuy = (g.h + 8 * g.vl - 1) / (8 * g.vl);
    for (int my = 0; my < mcuy && !o.overflow; ++my)
        for (int mx = 0; mx < mcux; ++mx)
            for (int c = 0; c < 3; ++c) {
                const int hs = c ? 1 : g.hl, vs = c ? 1 : g.vl, t = c ? 1 : 0;
                int prev = 0;
                for (int yy = 0; yy < vs; ++yy) {
                    const int by = my * vs + yy;
                    for (int xx = 0; xx < hs; ++xx) {
                        const int bx = mx * hs + xx;
                        const int16_t* blk;
                        if (by < g.bh[c] && bx < g.bw[c]) {
                            blk = coef + (g.cblk[c] + (long)by * g.bw[c] + bx) * 64;
                        } else {   // jccoefct.c dummy block: zero AC, DC of the previous block in the MCU
                            memset(dummy, 0, sizeof(dummy));
                            dummy[0] = (int16_t)prev;
                            blk = dummy;
                        }
                        encode_block(o, blk, last[c], T.dc[t], T.ac[t]);
                        prev = blk[0];
                    }
                }
            }
    o.flush();
    if (o.overflow || o.p + 2 > out + cap) return 0;
    *o.p++ = 0xFF;
    *o.p++ = 0xD9;
    return (size_t)(o.p - out);
}

}  // namespace

extern "C" int vd_jpeg_encode(vd_ctx* hctx, const uint8_t* frames, int n, int h, int w, size_t pitch, int where,
                              int quality, int subsampling, uint8_t* out, size_t cap, size_t* sizes) {
    Ctx* ctx = (Ctx*)hctx;
    if (!ctx) return vd_set_error(VD_ERR_ARG, "null context");
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (hipSetDevice(ctx->device) != hipSuccess) return vd_set_error(VD_ERR_HIP, "hipSetDevice(%d) failed", ctx->device);
    if (!frames || !out || !sizes || n <= 0 || n > ctx->cfg.max_batch || h <= 0 || w <= 0 || h > 65535 ||
        w > 65535 || pitch < (size_t)w * 3 || subsampling < 0 || subsampling > 2)
        return vd_set_error(VD_ERR_ARG, "vd_jpeg_encode: bad arguments");
    Geo g{};
    g.h = h; g.w = w;
    g.hl = subsampling == 0 ? 1 : 2;
    g.vl = subsampling == 2 ? 2 : 1;
    g.bpf = 0;
    for (int c = 0; c < 3; ++c) {   // width/height_in_blocks (jcmaster.c initial_setup)
        const int hs = c ? 1 : g.hl, vs = c ? 1 : g.vl;
        g.bw[c] = (w * hs + 8 * g.hl - 1) / (8 * g.hl);
        g.bh[c] = (h * vs + 8 * g.vl - 1) / (8 * g.vl);
        g.cblk[c] = g.bpf;
        g.bpf += (long)g.bw[c] * g.bh[c];
    }
    uint16_t ql[64], qc[64];
    quant_table(kStdLuma, quality, ql);
    quant_table(kStdChroma, quality, qc);
    // quantiser reciprocals [2][64] recip, [2][64] corr, [2][64] shift, natural order
    const size_t tab_bytes = 2 * 64 * 2 + 2 * 64 * 2 + 2 * 64;
    const size_t coef_bytes = (size_t)n * g.bpf * 128;
    int rc;
    if ((rc = ctx->ensure_staging(&ctx->jenc_dev, &ctx->jenc_dev_bytes, coef_bytes + tab_bytes + 64))) return rc;
    // pinned: the coefficients (host Huffman path), the quantiser tables, the device
    // path's code tables and its per-frame segment lengths
    const size_t pin_extra = 4 * 256 * 3 + (size_t)n * 4 + (size_t)(n + 1) * 8 + 64;
    if ((rc = ctx->ensure_pinned(&ctx->jenc_host, &ctx->jenc_host_bytes, coef_bytes + tab_bytes + pin_extra))) return rc;
    VD_CHECK_HIP(hipEventSynchronize(ctx->jpeg_ev));   // a previous H2D out of the pinned buffers is done
    uint8_t* hp = (uint8_t*)ctx->jenc_host + coef_bytes;
    uint16_t* hrecip = (uint16_t*)hp;
    uint16_t* hcorr = hrecip + 128;
    uint8_t* hshift = (uint8_t*)(hcorr + 128);
    for (int t = 0; t < 2; ++t)
        for (int k = 0; k < 64; ++k)
            reciprocal((t ? qc[k] : ql[k]) << 3, &hrecip[t * 64 + k], &hcorr[t * 64 + k], &hshift[t * 64 + k]);
    uint8_t* dp = (uint8_t*)ctx->jenc_dev;
    VD_CHECK_HIP(hipMemcpyAsync(dp + coef_bytes, hp, tab_bytes, hipMemcpyHostToDevice, ctx->stream));
    VD_CHECK_HIP(hipEventRecord(ctx->jpeg_ev, ctx->stream));
    const uint8_t* dframes = frames;
    if (where == VD_HOST) {
        if ((rc = ctx->ensure_staging(&ctx->stage_in, &ctx->stage_in_bytes, (size_t)n * h * pitch))) return rc;
        VD_CHECK_HIP(hipMemcpyAsync(ctx->stage_in, frames, (size_t)n * h * pitch, hipMemcpyHostToDevice, ctx->stream));
        dframes = (const uint8_t*)ctx->stage_in;
    }
    JpegEncArgs a{};
    a.src = dframes; a.pitch = pitch; a.n = n; a.h = h; a.w = w; a.hl = g.hl; a.vl = g.vl;
    for (int c = 0; c < 3; ++c) { a.bw[c] = g.bw[c]; a.bh[c] = g.bh[c]; a.cblk[c] = g.cblk[c]; }
    a.blocks_per_frame = g.bpf;
    a.recip = (const uint16_t*)(dp + coef_bytes);
    a.corr = a.recip + 128;
    a.shift = (const uint8_t*)(a.corr + 128);
    a.coef = (int16_t*)dp;
    ctx->t_begin(4, 0);
    hipError_t e = vd_launch_jpeg_fdct(a, ctx->stream);
    ctx->t_end();
    if (e != hipSuccess) return vd_set_error(VD_ERR_HIP, "jpeg fdct: %s", hipGetErrorString(e));
    if (ctx->tune.jenc_gpu) {
        // Huffman stage on the device (jpeg_enc.hip): segments land in device slots,
        // one D2H per frame of its stuffed length behind the host-written headers
        uint8_t hdr[1024];
        const size_t hl = write_headers(g, ql, qc, hdr);
        if (cap < hl + 2 + 16) return vd_set_error(VD_ERR_CAPACITY, "jpeg cap %zu below the headers", cap);
        const int mcux = (w + 8 * g.hl - 1) / (8 * g.hl), mcuy = (h + 8 * g.vl - 1) / (8 * g.vl);
        JpegHuffArgs ha{};
        ha.coef = a.coef; ha.blocks_per_frame = g.bpf; ha.n = n; ha.hl = g.hl; ha.vl = g.vl;
        for (int c = 0; c < 3; ++c) { ha.bw[c] = g.bw[c]; ha.bh[c] = g.bh[c]; ha.cblk[c] = g.cblk[c]; }
        ha.mcux = mcux;
        const long units = (long)mcux * mcuy * (g.hl * g.vl + 2);
        // 32-bit bit offsets: units x 1728 bits (the per-unit bound the word buffer is sized by) < 2^32
        if (units > 2000000) return vd_set_error(VD_ERR_ARG, "vd_jpeg_encode: frame too large for the device coder");
        ha.units = (int)units;
        ha.wcap = units * 54;                              // >= 1728 bits per unit: any block's codes fit
        ha.segcap = (long)(cap - hl - 2);
        const long nchunk_max = (ha.wcap * 4 + 4095) / 4096;
        const size_t huf_tab = 4 * 256 * 2 + 4 * 256;
        const size_t sz_bits = (size_t)n * units * 4, sz_words = (size_t)n * ha.wcap * 4, sz_seg = (size_t)n * ha.segcap;
        const size_t sz_ff = (size_t)n * nchunk_max * 4;
        const size_t need = huf_tab + sz_bits + (size_t)n * 8 + (size_t)(n + 1) * 8 + sz_ff + sz_words + sz_seg + 8 * 64;
        if ((rc = ctx->ensure_staging(&ctx->jhuf_dev, &ctx->jhuf_dev_bytes, need))) return rc;
        uint8_t* q = (uint8_t*)ctx->jhuf_dev;
        auto carve = [&](size_t bytes) { uint8_t* r = q; q += (bytes + 63) / 64 * 64; return r; };
        uint16_t* dcode = (uint16_t*)carve(huf_tab);
        ha.code = dcode; ha.size = (const uint8_t*)(dcode + 4 * 256);
        ha.bits = (unsigned*)carve(sz_bits);
        ha.total = (unsigned*)carve((size_t)n * 4);
        ha.segsize = (unsigned*)carve((size_t)n * 4);
        ha.segbase = (unsigned long long*)carve((size_t)(n + 1) * 8);
        ha.ffcnt = (unsigned*)carve(sz_ff);
        ha.words = (unsigned*)carve(sz_words);
        ha.seg = carve(sz_seg);
        // code / size tables [dc0, dc1, ac0, ac1] through the pinned buffer's tail
        const Tables& T = tables();
        uint16_t* htab = (uint16_t*)(hp + tab_bytes);
        const HuffEnc* order[4] = {&T.dc[0], &T.dc[1], &T.ac[0], &T.ac[1]};
        for (int k = 0; k < 4; ++k) {
            memcpy(htab + k * 256, order[k]->code, 512);
            memcpy((uint8_t*)(htab + 4 * 256) + k * 256, order[k]->size, 256);
        }
        VD_CHECK_HIP(hipMemcpyAsync(dcode, htab, huf_tab, hipMemcpyHostToDevice, ctx->stream));
        ctx->t_begin(4, 0);
        e = vd_launch_jpeg_huff(ha, ctx->stream);
        ctx->t_end();
        if (e != hipSuccess) return vd_set_error(VD_ERR_HIP, "jpeg huffman: %s", hipGetErrorString(e));
        // bit totals -> the chunk grid of the stuffing pass
        unsigned* htot = (unsigned*)(hp + tab_bytes + huf_tab);
        VD_CHECK_HIP(hipMemcpyAsync(htot, ha.total, (size_t)n * 4, hipMemcpyDeviceToHost, ctx->stream));
        VD_CHECK_HIP(hipStreamSynchronize(ctx->stream));
        unsigned maxbits = 0;
        std::vector<unsigned> htot_bits(htot, htot + n);
        for (int i = 0; i < n; ++i) maxbits = std::max(maxbits, htot[i]);
        ha.nchunk = (int)std::max<long>(1, ((long)maxbits / 8 + 1 + 4095) / 4096);
        if (ha.nchunk > nchunk_max) return vd_set_error(VD_ERR_HIP, "jpeg huffman: bit count past the buffer");
        ctx->t_begin(4, 0);
        e = vd_launch_jpeg_stuff(ha, ctx->stream);
        ctx->t_end();
        if (e != hipSuccess) return vd_set_error(VD_ERR_HIP, "jpeg stuffing: %s", hipGetErrorString(e));
        unsigned* hsz = htot;
        unsigned long long* hbase = (unsigned long long*)(hp + tab_bytes + huf_tab + (size_t)n * 4 + 8);
        hbase = (unsigned long long*)(((uintptr_t)hbase + 7) & ~(uintptr_t)7);
        VD_CHECK_HIP(hipMemcpyAsync(hsz, ha.segsize, (size_t)n * 4, hipMemcpyDeviceToHost, ctx->stream));
        VD_CHECK_HIP(hipMemcpyAsync(hbase, ha.segbase, (size_t)(n + 1) * 8, hipMemcpyDeviceToHost, ctx->stream));
        VD_CHECK_HIP(hipStreamSynchronize(ctx->stream));
        bool fits = true;
        for (int i = 0; i < n; ++i) fits = fits && hsz[i] != 0xFFFFFFFFu;
        if (!fits) {
            // sizes[] <- an upper bound of each frame's file (every coded byte stuffed):
            // the caller re-sizes its slots from it instead of guessing
            for (int i = 0; i < n; ++i) sizes[i] = hl + 2 + 2 * ((size_t)htot_bits[i] / 8 + 1) + 16;
            return vd_set_error(VD_ERR_CAPACITY, "jpeg frames do not fit %zu bytes (sizes[] holds the bound)", cap);
        }
        const size_t packed = (size_t)hbase[n];
        if ((rc = ctx->ensure_pinned(&ctx->jseg_host, &ctx->jseg_host_bytes, packed + 64))) return rc;
        VD_CHECK_HIP(hipMemcpyAsync(ctx->jseg_host, ha.seg, packed, hipMemcpyDeviceToHost, ctx->stream));
        VD_CHECK_HIP(hipStreamSynchronize(ctx->stream));
        // headers + segment + EOI into the caller's slots, host threads over frames
        const uint8_t* segs = (const uint8_t*)ctx->jseg_host;
        std::atomic<int> nx{0};
        auto copier = [&]() {
            for (int i; (i = nx.fetch_add(1)) < n;) {
                uint8_t* o = out + (size_t)i * cap;
                memcpy(o, hdr, hl);
                memcpy(o + hl, segs + hbase[i], hsz[i]);
                o[hl + hsz[i]] = 0xFF;
                o[hl + hsz[i] + 1] = 0xD9;
                sizes[i] = hl + hsz[i] + 2;
            }
        };
        const int nth = std::max(1, std::min(n, ctx->jpeg_threads));
        std::vector<std::thread> cp;
        for (int t = 1; t < nth; ++t) cp.emplace_back(copier);
        copier();
        for (auto& t : cp) t.join();
        return VD_OK;
    }
    VD_CHECK_HIP(hipMemcpyAsync(ctx->jenc_host, dp, coef_bytes, hipMemcpyDeviceToHost, ctx->stream));
    VD_CHECK_HIP(hipStreamSynchronize(ctx->stream));
    // Huffman stage, one frame per host thread
    const int16_t* hc = (const int16_t*)ctx->jenc_host;
    std::atomic<int> next{0};
    auto worker = [&]() {
        for (int i; (i = next.fetch_add(1)) < n;)
            sizes[i] = encode_frame(g, hc + (size_t)i * g.bpf * 64, ql, qc, out + (size_t)i * cap, cap);
    };
    const int nthreads = std::max(1, std::min(n, ctx->jpeg_threads));
    std::vector<std::thread> pool;
    for (int t = 1; t < nthreads; ++t) pool.emplace_back(worker);
    worker();
    for (auto& t : pool) t.join();
    for (int i = 0; i < n; ++i)
        if (!sizes[i]) return vd_set_error(VD_ERR_CAPACITY, "jpeg frame %d does not fit %zu bytes", i, cap);
    return VD_OK;
}
