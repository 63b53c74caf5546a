// pre.hip — letterbox/normalise/pack, max-pool and nearest-upsample kernels.
//
// letterbox_kernel replaces, in one HBM pass per frame batch:
//   Retinaface.preprocess (detect_face/face.py:65-88) = letterbox_image
//   (detect_face/utils/utils.py:8-18: cv2.resize INTER_LINEAR [ext] + paste in a
//   128-filled canvas) + preprocess_input (:27-28, subtract (104,117,123) in
//   RGB order) + HWC->CHW + float32 + H2D; and the ultralytics LetterBox
//   (stride-32 auto padding, value 114, BGR<->RGB flip, /255) [ext] of the plate
//   detector call (combine_detect.py:217). Output is NHWC with `cpad` channels
//   (3 real + zeros) so the stem conv reads one 16-byte vector per tap.
//   cv2.resize rounding is restated exactly (oracle/letterbox.py):
//     COPY  (dsize == ssize), AREA2 (exact 2x: (a+b+c+d+2)>>2),
//     LINEAR (11-bit fixed point, SIMD vertical form).
#include "vd_common.h"
#include "vd_math.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>

namespace {

struct Tap { int s0, s1, a0, a1; };

__device__ __forceinline__ Tap linear_tap(int d, int ssize, double scale) {
    // fx = (float)((dx + 0.5) * scale_x - 0.5); sx = floor(fx); fx -= sx; border clamps
    float f = (float)VD_DSUB(VD_DMUL(VD_DADD((double)d, 0.5), scale), 0.5);
    int s = (int)floorf(f);
    f = VD_FSUB(f, (float)s);
    if (s < 0) { f = 0.f; s = 0; }
    if (s >= ssize - 1) { f = 0.f; s = ssize - 1; }
    Tap t;
    t.s0 = s;
    t.s1 = min(s + 1, ssize - 1);
    t.a0 = __float2int_rn(VD_FMUL(VD_FSUB(1.0f, f), 2048.0f));
    t.a1 = __float2int_rn(VD_FMUL(f, 2048.0f));
    return t;
}

// The 3 channels of resized pixel (y, x) (interpolation taps computed once).
__device__ __forceinline__ void resized_px3(const LetterboxArgs& a, const uint8_t* img, int y, int x, int out[3]) {
    if (a.mode == LB_COPY) {
        const uint8_t* p = img + (size_t)y * a.pitch + x * 3;
        out[0] = p[0]; out[1] = p[1]; out[2] = p[2];
        return;
    }
    if (a.mode == LB_AREA2) {
        const uint8_t* p = img + (size_t)(2 * y) * a.pitch + (2 * x) * 3;
#pragma unroll
        for (int c = 0; c < 3; ++c) out[c] = (p[c] + p[c + 3] + p[a.pitch + c] + p[a.pitch + c + 3] + 2) >> 2;
        return;
    }
    const Tap tx = linear_tap(x, a.iw, a.scale_x);
    const Tap ty = linear_tap(y, a.ih, a.scale_y);
    const uint8_t* r0 = img + (size_t)ty.s0 * a.pitch;
    const uint8_t* r1 = img + (size_t)ty.s1 * a.pitch;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        int d0 = r0[tx.s0 * 3 + c] * tx.a0 + r0[tx.s1 * 3 + c] * tx.a1;
        int d1 = r1[tx.s0 * 3 + c] * tx.a0 + r1[tx.s1 * 3 + c] * tx.a1;
        int v = ((((d0 >> 4) * ty.a0) >> 16) + (((d1 >> 4) * ty.a1) >> 16) + 2) >> 2;
        out[c] = v < 0 ? 0 : (v > 255 ? 255 : v);
    }
}

// Normalised canvas pixel (y, x) (resized image or pad value), 3 channels.
__device__ __forceinline__ void canvas_px(const LetterboxArgs& a, const uint8_t* img, int y, int x, float v[3]) {
    const int ry = y - a.top, rx = x - a.left;
    const bool inside = (unsigned)ry < (unsigned)a.nh && (unsigned)rx < (unsigned)a.nw;
    int p3[3] = {0, 0, 0};
    if (inside) resized_px3(a, img, ry, rx, p3);
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const int pv = a.flip ? p3[2 - c] : p3[c];
        const float px = inside ? (float)pv : a.pad_value;
        v[c] = VD_FDIV(VD_FSUB(px, a.mean[c]), a.div);
    }
}

// one 2x2 block's 16 values (4 sub-pixels x [3 channels, 0]): bf16, fp16 (a.out_f16:
// the fp32 plan's fused face stem canvas, integer values, exact) or f32 (a.out_f32)
__device__ __forceinline__ void store_s2d(const LetterboxArgs& a, size_t idx, const float (&v)[16]) {
    if (a.out_f32) {   // the fp32 plan's plate canvas: integer values as f32, 64 B per block
        float4* o = (float4*)((float*)a.out + idx * 16);
#pragma unroll
        for (int i = 0; i < 4; ++i) o[i] = make_float4(v[4 * i], v[4 * i + 1], v[4 * i + 2], v[4 * i + 3]);
        return;
    }
    uint4 u[2];
    if (a.out_f16) {
        _Float16 t[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) t[i] = (_Float16)v[i];
        u[0] = *(const uint4*)t; u[1] = *(const uint4*)(t + 8);
    } else {
        __bf16 t[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) t[i] = (__bf16)v[i];
        u[0] = *(const uint4*)t; u[1] = *(const uint4*)(t + 8);
    }
    uint4* out = (uint4*)((uint16_t*)a.out + idx * 16);
    out[0] = u[0];
    out[1] = u[1];
}

// Space-to-depth form (a.s2d): one thread per 2x2 canvas block, 32 B out.
__global__ __launch_bounds__(256) void letterbox_s2d_kernel(LetterboxArgs a) {
    const int X = blockIdx.x * 256 + threadIdx.x;
    const int Y = blockIdx.y;
    const int f = blockIdx.z;
    const int OW = a.ow / 2 + 1, OH = a.oh / 2 + 1;
    if (X >= OW) return;
    const uint8_t* img = a.src + (size_t)f * a.ih * a.pitch;
    float t[16];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        const int y = 2 * Y + (s >> 1) - 1, x = 2 * X + (s & 1) - 1;
        float v[3] = {0.f, 0.f, 0.f};   // conv zero padding outside the canvas
        if ((unsigned)y < (unsigned)a.oh && (unsigned)x < (unsigned)a.ow) canvas_px(a, img, y, x, v);
        t[4 * s + 0] = v[0]; t[4 * s + 1] = v[1]; t[4 * s + 2] = v[2];
        t[4 * s + 3] = 0.f;
    }
    store_s2d(a, ((size_t)f * OH + Y) * OW + X, t);
}

// Space-to-depth form with the source rows staged in LDS: one workgroup per
// (frame, X' row Y) loads the <= 4 source rows its two canvas rows interpolate from
// with 16-B loads (only rows some output reads: 2 of every 3 at 1080p -> 360), then
// every 2x2 block is computed from LDS. Same arithmetic as resized_px3 / canvas_px.
constexpr int LB_LDS_MAX = 16384;   // max bytes per staged source row (frames up to 5461 px wide)

__device__ __forceinline__ void lb_src_rows(const LetterboxArgs& a, int y, int* r0, int* r1, Tap* ty, bool* inside) {
    const int ry = y - a.top;
    *inside = (unsigned)y < (unsigned)a.oh && (unsigned)ry < (unsigned)a.nh;
    *r0 = *r1 = -1;
    if (!*inside) return;
    if (a.mode == LB_COPY) { *r0 = *r1 = ry; return; }
    if (a.mode == LB_AREA2) { *r0 = 2 * ry; *r1 = 2 * ry + 1; return; }
    *ty = linear_tap(ry, a.ih, a.scale_y);
    *r0 = ty->s0;
    // a zero-weight second row (an exact gather: 1080p -> 640 samples rows 3y + 1 with weights
    // (1, 0)) adds exact zeros, so it is not staged: the pixel reads row r0 twice instead
    *r1 = ty->a1 ? ty->s1 : -1;
}

__device__ __forceinline__ void lb_px_lds(const LetterboxArgs& a, const uint8_t* L0, const uint8_t* L1, const Tap& ty,
                                          int x, bool row_in, float v[3]) {
    const int rx = x - a.left;
    const bool inside = row_in && (unsigned)rx < (unsigned)a.nw;
    int p3[3] = {0, 0, 0};
    if (inside) {
        if (a.mode == LB_COPY) {
#pragma unroll
            for (int c = 0; c < 3; ++c) p3[c] = L0[rx * 3 + c];
        } else if (a.mode == LB_AREA2) {
#pragma unroll
            for (int c = 0; c < 3; ++c)
                p3[c] = (L0[6 * rx + c] + L0[6 * rx + c + 3] + L1[6 * rx + c] + L1[6 * rx + c + 3] + 2) >> 2;
        } else if (a.gx_k > 0 && ty.a1 == 0) {
            // exact gather both ways (weights (1, 0): the bilinear sum below reduces to the
            // source byte exactly, ((4 p + 2) >> 2) = p), e.g. 1080p -> 640: column 3 rx + 1
            const int sx = a.gx_k * rx + a.gx_c;
#pragma unroll
            for (int c = 0; c < 3; ++c) p3[c] = L0[sx * 3 + c];
        } else {
            const Tap tx = linear_tap(rx, a.iw, a.scale_x);
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                const int d0 = L0[tx.s0 * 3 + c] * tx.a0 + L0[tx.s1 * 3 + c] * tx.a1;
                const int d1 = L1[tx.s0 * 3 + c] * tx.a0 + L1[tx.s1 * 3 + c] * tx.a1;
                const int q = ((((d0 >> 4) * ty.a0) >> 16) + (((d1 >> 4) * ty.a1) >> 16) + 2) >> 2;
                p3[c] = q < 0 ? 0 : (q > 255 ? 255 : q);
            }
        }
    }
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const int pv = a.flip ? p3[2 - c] : p3[c];
        const float px = inside ? (float)pv : a.pad_value;
        v[c] = VD_FDIV(VD_FSUB(px, a.mean[c]), a.div);
    }
}

__global__ __launch_bounds__(256) void letterbox_s2d_lds_kernel(LetterboxArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lrow[];   // 4 staged rows of RS bytes
    const int Y = blockIdx.x, f = blockIdx.y;
    const int OW = a.ow / 2 + 1, OH = a.oh / 2 + 1;
    const uint8_t* img = a.src + (size_t)f * a.ih * a.pitch;
    int rows[4];
    Tap ty[2];
    bool rin[2];
    lb_src_rows(a, 2 * Y - 1, &rows[0], &rows[1], &ty[0], &rin[0]);
    lb_src_rows(a, 2 * Y, &rows[2], &rows[3], &ty[1], &rin[1]);
    const int rb = a.iw * 3;
    const int nch = (rb + 15) / 16;
    const int RS = nch * 16;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        if (rows[k] < 0) continue;
        const uint8_t* src = img + (size_t)rows[k] * a.pitch;
        uint8_t* dst = lrow + k * RS;
        if (((uintptr_t)src & 15) == 0) {
            for (int i = threadIdx.x; i < nch; i += 256) {
                if (16 * i + 16 <= rb) *(uint4*)(dst + 16 * i) = *(const uint4*)(src + 16 * i);
                else for (int b = 16 * i; b < rb; ++b) dst[b] = src[b];
            }
        } else {
            for (int i = threadIdx.x; i < rb; i += 256) dst[i] = src[i];
        }
    }
    __syncthreads();
    for (int X = threadIdx.x; X < OW; X += 256) {
        float t[16];
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const int h = s >> 1;
            const int x = 2 * X + (s & 1) - 1;
            float v[3] = {0.f, 0.f, 0.f};   // conv zero padding outside the canvas
            const int y = 2 * Y + h - 1;
            if ((unsigned)y < (unsigned)a.oh && (unsigned)x < (unsigned)a.ow)
                lb_px_lds(a, lrow + (2 * h) * RS, lrow + (2 * h + (rows[2 * h + 1] >= 0 ? 1 : 0)) * RS, ty[h], x, rin[h], v);
            t[4 * s + 0] = v[0]; t[4 * s + 1] = v[1]; t[4 * s + 2] = v[2];
            t[4 * s + 3] = 0.f;
        }
        store_s2d(a, ((size_t)f * OH + Y) * OW + X, t);
    }
}

// Two space-to-depth canvases of the same frames in one pass (the face and the
// plate letterbox of vd_process): both resize to the same nw x nh with the same
// filter, so a source row feeds block row Y of canvas a and block row Y - dY of
// canvas b; each source row is staged once and both canvases are written from it.
// Per pixel the arithmetic is exactly letterbox_s2d_lds_kernel's for each canvas.
// Block rows Y run over the union [y0, y0 + gridDim.x), X over [x0, x0 + nx).
__global__ __launch_bounds__(256) void letterbox_s2d_pair_kernel(LetterboxArgs a, LetterboxArgs b, int dY, int dX,
                                                                 int y0, int x0, int nx) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lrow[];
    const int Y = y0 + (int)blockIdx.x, f = blockIdx.y;
    const int Yb = Y - dY;
    const int OWa = a.ow / 2 + 1, OHa = a.oh / 2 + 1, OWb = b.ow / 2 + 1, OHb = b.oh / 2 + 1;
    const bool ya = (unsigned)Y < (unsigned)OHa, yb = (unsigned)Yb < (unsigned)OHb;
    const uint8_t* img = a.src + (size_t)f * a.ih * a.pitch;
    int ra[4] = {-1, -1, -1, -1}, rb[4] = {-1, -1, -1, -1};
    Tap tya[2], tyb[2];
    bool rina[2] = {false, false}, rinb[2] = {false, false};
    if (ya) {
        lb_src_rows(a, 2 * Y - 1, &ra[0], &ra[1], &tya[0], &rina[0]);
        lb_src_rows(a, 2 * Y, &ra[2], &ra[3], &tya[1], &rina[1]);
    }
    if (yb) {
        lb_src_rows(b, 2 * Yb - 1, &rb[0], &rb[1], &tyb[0], &rinb[0]);
        lb_src_rows(b, 2 * Yb, &rb[2], &rb[3], &tyb[1], &rinb[1]);
    }
    const int rbytes = a.iw * 3;
    const int nch = (rbytes + 15) / 16;
    const int RS = nch * 16;
    const bool st1[2] = {ra[1] >= 0 || rb[1] >= 0, ra[3] >= 0 || rb[3] >= 0};   // second rows staged
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int row = ra[k] >= 0 ? ra[k] : rb[k];   // the same source row when both canvases need one
        if (row < 0) continue;
        const uint8_t* src = img + (size_t)row * a.pitch;
        uint8_t* dst = lrow + k * RS;
        if (((uintptr_t)src & 15) == 0) {
            for (int i = threadIdx.x; i < nch; i += 256) {
                if (16 * i + 16 <= rbytes) *(uint4*)(dst + 16 * i) = *(const uint4*)(src + 16 * i);
                else for (int q = 16 * i; q < rbytes; ++q) dst[q] = src[q];
            }
        } else {
            for (int i = threadIdx.x; i < rbytes; i += 256) dst[i] = src[i];
        }
    }
    __syncthreads();
    for (int X = x0 + (int)threadIdx.x; X < x0 + nx; X += 256) {
#pragma unroll
        for (int cv = 0; cv < 2; ++cv) {
            const LetterboxArgs& c = cv ? b : a;
            const int XX = cv ? X - dX : X, YY = cv ? Yb : Y;
            if (!(cv ? yb : ya) || (unsigned)XX >= (unsigned)(cv ? OWb : OWa)) continue;
            const Tap* ty = cv ? tyb : tya;
            const bool* rin = cv ? rinb : rina;
            float t[16];
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const int h = s >> 1;
                const int x = 2 * XX + (s & 1) - 1;
                float v[3] = {0.f, 0.f, 0.f};
                const int y = 2 * YY + h - 1;
                if ((unsigned)y < (unsigned)c.oh && (unsigned)x < (unsigned)c.ow)
                    lb_px_lds(c, lrow + (2 * h) * RS, lrow + (2 * h + (st1[h] ? 1 : 0)) * RS, ty[h], x, rin[h], v);
                t[4 * s + 0] = v[0]; t[4 * s + 1] = v[1]; t[4 * s + 2] = v[2];
                t[4 * s + 3] = 0.f;
            }
            store_s2d(c, ((size_t)f * (cv ? OHb : OHa) + YY) * (cv ? OWb : OWa) + XX, t);   // bf16, fp16 or f32
        }
    }
}

__global__ __launch_bounds__(256) void letterbox_kernel(LetterboxArgs a) {
    const int x = blockIdx.x * 256 + threadIdx.x;
    const int y = blockIdx.y;
    const int f = blockIdx.z;
    if (x >= a.ow) return;
    const uint8_t* img = a.src + (size_t)f * a.ih * a.pitch;
    float v[3];
    canvas_px(a, img, y, x, v);
    const size_t o = (((size_t)f * a.oh + y) * a.ow + x) * a.cpad;
    if (a.out_f32) {
        float* out = (float*)a.out + o;
        float4 w0 = make_float4(v[0], v[1], v[2], 0.f);
        *(float4*)out = w0;
        for (int c = 4; c < a.cpad; c += 4) *(float4*)(out + c) = make_float4(0.f, 0.f, 0.f, 0.f);
    } else if (a.out_f16) {   // integers in [-123, 151]: exact in fp16 as in bf16
        _Float16* out = (_Float16*)a.out + o;
        _Float16 tmp[8];
        tmp[0] = (_Float16)v[0]; tmp[1] = (_Float16)v[1]; tmp[2] = (_Float16)v[2];
        for (int c = 3; c < 8; ++c) tmp[c] = (_Float16)0.f;
        *(uint4*)out = *(const uint4*)tmp;
        for (int c = 8; c < a.cpad; c += 8) *(uint4*)(out + c) = make_uint4(0, 0, 0, 0);
    } else {
        __bf16* out = (__bf16*)a.out + o;
        __bf16 tmp[8];
        tmp[0] = (__bf16)v[0]; tmp[1] = (__bf16)v[1]; tmp[2] = (__bf16)v[2];
        for (int c = 3; c < 8; ++c) tmp[c] = (__bf16)0.f;
        *(uint4*)out = *(const uint4*)tmp;
        for (int c = 8; c < a.cpad; c += 8) *(uint4*)(out + c) = make_uint4(0, 0, 0, 0);
    }
}

// NHWC max-pool (torch semantics: padded taps ignored), vectorised 16 B per thread.
template <typename T>
__global__ __launch_bounds__(256) void maxpool_kernel(const T* x, int xh, int xw, int ldx, int xcoff,
                                                      T* y, int yh, int yw, int ldy, int ycoff,
                                                      int c, int k, int s, int p, int total) {
    constexpr int VEC = 16 / sizeof(T);
    const int idx = blockIdx.x * 256 + threadIdx.x;
    if (idx >= total) return;
    const int cv = c / VEC;
    const int ci = (idx % cv) * VEC;
    int pix = idx / cv;
    const int ox = pix % yw; pix /= yw;
    const int oy = pix % yh;
    const int b = pix / yh;
    float m[VEC];
#pragma unroll
    for (int e = 0; e < VEC; ++e) m[e] = -__builtin_huge_valf();
    for (int dy = 0; dy < k; ++dy) {
        int iy = oy * s - p + dy;
        if ((unsigned)iy >= (unsigned)xh) continue;
        for (int dx = 0; dx < k; ++dx) {
            int ix = ox * s - p + dx;
            if ((unsigned)ix >= (unsigned)xw) continue;
            uint4 u = *(const uint4*)(x + (((size_t)b * xh + iy) * xw + ix) * ldx + xcoff + ci);
            const T* t = (const T*)&u;
#pragma unroll
            for (int e = 0; e < VEC; ++e) m[e] = fmaxf(m[e], (float)t[e]);
        }
    }
    T o[VEC];
#pragma unroll
    for (int e = 0; e < VEC; ++e) o[e] = (T)m[e];
    *(uint4*)(y + (((size_t)b * yh + oy) * yw + ox) * ldy + ycoff + ci) = *(const uint4*)o;
}

// Nearest 2x upsample into a channel slice (ultralytics nn.Upsample + Concat).
template <typename T>
__global__ __launch_bounds__(256) void upsample2x_kernel(const T* x, int xh, int xw, int ldx, int xcoff,
                                                         T* y, int ldy, int ycoff, int c, int total) {
    constexpr int VEC = 16 / sizeof(T);
    const int idx = blockIdx.x * 256 + threadIdx.x;
    if (idx >= total) return;
    const int cv = c / VEC;
    const int ci = (idx % cv) * VEC;
    int pix = idx / cv;
    const int yw = 2 * xw, yh = 2 * xh;
    const int ox = pix % yw; pix /= yw;
    const int oy = pix % yh;
    const int b = pix / yh;
    uint4 u = *(const uint4*)(x + (((size_t)b * xh + (oy >> 1)) * xw + (ox >> 1)) * ldx + xcoff + ci);
    *(uint4*)(y + (((size_t)b * yh + oy) * yw + ox) * ldy + ycoff + ci) = u;
}

}  // namespace

// Same frames, both 16-bit (bf16 / fp16) space-to-depth canvases, the same resize
// (nw, nh, filter) and even relative offsets of the pasted images.
bool vd_letterbox_pair_ok(const LetterboxArgs& a, const LetterboxArgs& b) {
    return a.s2d && b.s2d && a.src == b.src && a.n == b.n &&
           a.ih == b.ih && a.iw == b.iw && a.pitch == b.pitch && a.iw * 3 <= LB_LDS_MAX && a.nw == b.nw &&
           a.nh == b.nh && a.mode == b.mode && a.scale_x == b.scale_x && a.scale_y == b.scale_y &&
           ((a.top - b.top) & 1) == 0 && ((a.left - b.left) & 1) == 0;
}

// linear_tap on the host (the same IEEE round-to-nearest operations as the device): source
// column s0 and second weight a1 of resized column d
static void lb_tap_host(int d, int ssize, double scale, int* s0, int* a1) {
    float f = (float)((((double)d + 0.5) * scale) - 0.5);
    int s = (int)std::floor(f);
    f = f - (float)s;
    if (s < 0) { f = 0.f; s = 0; }
    if (s >= ssize - 1) { f = 0.f; s = ssize - 1; }
    *s0 = s;
    *a1 = (int)std::nearbyint(f * 2048.0f);
}

// LB_LINEAR columns that are an exact affine gather (every a1 = 0, s0 = k d + c): the kernels'
// gather fast path (checked over every resized column, so it is exact by construction)
static void lb_set_gather(LetterboxArgs& a) {
    a.gx_k = a.gx_c = 0;
    if (a.mode != LB_LINEAR || a.nw < 2) return;
    int s0, s1, a1;
    lb_tap_host(0, a.iw, a.scale_x, &s0, &a1);
    lb_tap_host(1, a.iw, a.scale_x, &s1, &a1);
    const int k = s1 - s0, c = s0;
    if (k <= 0) return;
    for (int d = 0; d < a.nw; ++d) {
        lb_tap_host(d, a.iw, a.scale_x, &s0, &a1);
        if (a1 != 0 || s0 != k * d + c) return;
    }
    a.gx_k = k;
    a.gx_c = c;
}

hipError_t vd_launch_letterbox_pair(const LetterboxArgs& a0, const LetterboxArgs& b0, hipStream_t s) {
    LetterboxArgs a = a0, b = b0;
    lb_set_gather(a);
    lb_set_gather(b);
    if (!vd_letterbox_pair_ok(a, b)) return hipErrorInvalidValue;
    static const bool attr = [] {
        (void)hipFuncSetAttribute((const void*)letterbox_s2d_pair_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  4 * LB_LDS_MAX);
        return true;
    }();
    (void)attr;
    const int dY = (a.top - b.top) / 2, dX = (a.left - b.left) / 2;
    const int y0 = std::min(0, dY), y1 = std::max(a.oh / 2 + 1, b.oh / 2 + 1 + dY);
    const int x0 = std::min(0, dX), x1 = std::max(a.ow / 2 + 1, b.ow / 2 + 1 + dX);
    const size_t lds = 4 * (size_t)((a.iw * 3 + 15) / 16 * 16);
    hipLaunchKernelGGL(letterbox_s2d_pair_kernel, dim3(y1 - y0, a.n), dim3(256), lds, s, a, b, dY, dX, y0, x0, x1 - x0);
    return hipGetLastError();
}

hipError_t vd_launch_letterbox(const LetterboxArgs& a0, hipStream_t s) {
    LetterboxArgs a = a0;
    lb_set_gather(a);
    if (a.s2d && a.iw * 3 <= LB_LDS_MAX) {
        static const bool attr = [] {
            (void)hipFuncSetAttribute((const void*)letterbox_s2d_lds_kernel,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 4 * LB_LDS_MAX);
            return true;
        }();
        (void)attr;
        const size_t lds = 4 * (size_t)((a.iw * 3 + 15) / 16 * 16);
        dim3 grid(a.oh / 2 + 1, a.n);
        hipLaunchKernelGGL(letterbox_s2d_lds_kernel, grid, dim3(256), lds, s, a);
        return hipGetLastError();
    }
    if (a.s2d) {
        dim3 grid((a.ow / 2 + 1 + 255) / 256, a.oh / 2 + 1, a.n);
        hipLaunchKernelGGL(letterbox_s2d_kernel, grid, dim3(256), 0, s, a);
        return hipGetLastError();
    }
    dim3 grid((a.ow + 255) / 256, a.oh, a.n);
    hipLaunchKernelGGL(letterbox_kernel, grid, dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t vd_launch_maxpool(bool f32, bool f16, const void* x, int n, int xh, int xw, int ldx, int xcoff,
                             void* y, int yh, int yw, int ldy, int ycoff, int c, int k, int st, int p,
                             hipStream_t s) {
    const int vec = f32 ? 4 : 8;
    const int total = n * yh * yw * (c / vec);
    dim3 grid((total + 255) / 256);
    if (f32)
        hipLaunchKernelGGL(maxpool_kernel<float>, grid, dim3(256), 0, s, (const float*)x, xh, xw, ldx, xcoff,
                           (float*)y, yh, yw, ldy, ycoff, c, k, st, p, total);
    else if (f16)
        hipLaunchKernelGGL(maxpool_kernel<_Float16>, grid, dim3(256), 0, s, (const _Float16*)x, xh, xw, ldx, xcoff,
                           (_Float16*)y, yh, yw, ldy, ycoff, c, k, st, p, total);
    else
        hipLaunchKernelGGL(maxpool_kernel<__bf16>, grid, dim3(256), 0, s, (const __bf16*)x, xh, xw, ldx, xcoff,
                           (__bf16*)y, yh, yw, ldy, ycoff, c, k, st, p, total);
    return hipGetLastError();
}

// (a pure copy: the bf16 instantiation moves fp16 bits unchanged)
hipError_t vd_launch_upsample2x(bool f32, const void* x, int n, int xh, int xw, int ldx, int xcoff,
                                void* y, int ldy, int ycoff, int c, hipStream_t s) {
    const int vec = f32 ? 4 : 8;
    const int total = n * 4 * xh * xw * (c / vec);
    dim3 grid((total + 255) / 256);
    if (f32)
        hipLaunchKernelGGL(upsample2x_kernel<float>, grid, dim3(256), 0, s, (const float*)x, xh, xw, ldx, xcoff,
                           (float*)y, ldy, ycoff, c, total);
    else
        hipLaunchKernelGGL(upsample2x_kernel<__bf16>, grid, dim3(256), 0, s, (const __bf16*)x, xh, xw, ldx, xcoff,
                           (__bf16*)y, ldy, ycoff, c, total);
    return hipGetLastError();
}
