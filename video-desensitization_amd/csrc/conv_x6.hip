// conv_x6.hip — fp32 convolution on the bf16 matrix cores by exact operand
// decomposition (VD_PREC_FP32 with option f32_split = 1, the default).
//
// Every f32 operand is split EXACTLY into three bf16 terms, x = x0 + x1 + x2
// (x0 = the top 8 significand bits, x1 the next 8, x2 the last 8: each residual
// is exact in f32 and fits the next term), and the product is the sum of the six
// cross terms with i + j <= 2:
//     a*b ~= a0 b0 + a0 b1 + a1 b0 + a0 b2 + a1 b1 + a2 b0
// Each term is an exact 16-bit product accumulated in f32 by
// v_mfma_f32_16x16x32_bf16; the dropped terms (a1 b2, a2 b1, a2 b2) are below
// 2^-22 |ab|, so a K-long dot product carries the same error as an f32 fma chain
// (measured in tests/test_gpu_kernels.py against float64: error at the level of
// the exact-f32 MFMA path). Six bf16 MFMAs (96 cycles per 16x16x32 block) replace
// eight exact-f32 v_mfma_f32_16x16x4_f32 (256 cycles): 2.67x the f32 MFMA rate.
//
// Same conv contract as conv.hip (NHWC f32 activations, K = (kh, kw, c) with c
// fastest, fused BN scale/shift + residual + activation, channel-sliced
// in/out); replaces the same reference layers (retinaface.py:71-92 via
// torchvision resnet50 [ext], layers.py:10-114, the YOLOv8n convs).
//
// Schedule: 256 x 128 tile (M pixels x N channels), 8 waves (4 x 2, each a
// 64 x 64 wave tile of 16 MFMA blocks), K tile 32, two LDS stages of
// {A planes 3 x 256 x 64 B, B planes 3 x 128 x 64 B} = 72 KB each.
//   * A (f32 pixels): global -> registers (two 16-B loads per 8 k), split by
//     bit masking + exact f32 subtraction, written as three 16-B bf16 chunks;
//     loads for tile t+2 are issued while tile t computes.
//   * B (weights): split once at weight load into [Npad][Kpad/32][3 planes][32]
//     bf16; LDS-DMA straight into the stage (source-side swizzle).
//   * 64-B LDS rows, chunk' = chunk ^ (((row >> 3) & 1) * 3): conflict-free
//     ds_read_b128 fragment reads for the 16-row MFMA operand pattern.
#include "vd_common.h"
#include <algorithm>
#include <type_traits>
#include <cmath>
#include <cstring>

namespace {

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void_t;

constexpr int KT = 32;                          // K per tile (one bf16 MFMA k-step)
constexpr int kAmaxFrames = 1024;               // LDS reserved for per-frame max slots (frames per launch)

// Two forms: the big tile (256 x BN, 8 waves, two LDS stages, one workgroup per CU)
// for the compute-heavy layers, and the small tile (128 x BN, 4 waves, ONE stage,
// three workgroups per CU) for small-K / small-M layers, where a workgroup's
// load -> compute -> epilogue phases are short and neighbours on the CU overlap them.
// TERMS: 3 = bf16 triples (A and B), 2 = fp16 pairs (A and B), 1 = fp16 pair weights
// with activations exact in fp16 (one A plane: the integer-valued face canvas)
template <int BM_, int BN, int NT_, int NST, int TERMS, int MF = 16> struct X6Shape {
    static constexpr int TA = TERMS == 1 ? 1 : TERMS, TB = TERMS == 1 ? 2 : TERMS;   // A / B planes
    static constexpr int BM = BM_, BNV = BN, NT = NT_, WAVES = NT / 64, TERMSV = TERMS;
    static constexpr int PL_A = BM * 64;                       // bytes per A plane
    static constexpr int PL_B = BN * 64;                       // bytes per B plane
    static constexpr int STAGE = TA * PL_A + TB * PL_B;        // 256 x 128: 73 728 B (3 terms), 49 152 B (2)
    static constexpr int EPR = NST == 2 ? 128 : 64;            // epilogue rows per pass
    static constexpr int EPLD = BN + 4;                        // f32 epilogue row stride
    static constexpr int LDS = NST * STAGE > EPR * EPLD * 4 ? NST * STAGE : EPR * EPLD * 4;
    static constexpr int WAVES_N = BN >= 64 ? 2 : 1;
    static constexpr int WAVES_M = WAVES / WAVES_N;
    static constexpr int WTM = BM / WAVES_M, WTN = BN / WAVES_N;
    static constexpr int TM = WTM / MF, TN = WTN / MF;            // MFMA blocks per wave tile
    static constexpr int NDMA = TB * BN / 16;                  // 1-KB DMA instructions per K tile
    static constexpr int AROWS = NT / 4;                       // A rows per staging pass
    static constexpr int AITEMS = BM / AROWS;                  // A items (row, 8 k) per thread: 2 (8 waves), 4 (4 waves)
    static_assert(BM % AROWS == 0 && (AITEMS == 2 || AITEMS == 4), "A items per thread");
};

__device__ __forceinline__ int swz(int row, int chunk) { return row * 64 + ((chunk ^ (((row >> 3) & 1) * 3)) << 4); }

// s_waitcnt vmcnt(n) for n in [0, 23] (immediate operand)
__device__ __forceinline__ void wait_vm(int n) {
    switch (n) {
        case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); return;
        case 9: asm volatile("s_waitcnt vmcnt(9)" ::: "memory"); return;
        case 10: asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); return;
        case 11: asm volatile("s_waitcnt vmcnt(11)" ::: "memory"); return;
        case 12: asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); return;
        case 13: asm volatile("s_waitcnt vmcnt(13)" ::: "memory"); return;
        case 14: asm volatile("s_waitcnt vmcnt(14)" ::: "memory"); return;
        case 15: asm volatile("s_waitcnt vmcnt(15)" ::: "memory"); return;
        case 16: asm volatile("s_waitcnt vmcnt(16)" ::: "memory"); return;
        case 17: asm volatile("s_waitcnt vmcnt(17)" ::: "memory"); return;
        case 18: asm volatile("s_waitcnt vmcnt(18)" ::: "memory"); return;
        case 19: asm volatile("s_waitcnt vmcnt(19)" ::: "memory"); return;
        case 20: asm volatile("s_waitcnt vmcnt(20)" ::: "memory"); return;
        case 21: asm volatile("s_waitcnt vmcnt(21)" ::: "memory"); return;
        case 22: asm volatile("s_waitcnt vmcnt(22)" ::: "memory"); return;
        case 23: asm volatile("s_waitcnt vmcnt(23)" ::: "memory"); return;
        default: break;
    }
    switch (n < 8 ? n : 7) {
        case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
        case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
        case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
        case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
        case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
        case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
        case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
        default: asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); break;
    }
}

// s_waitcnt vmcnt(N) for a compile-time N (no branch tree)
template <int N>
__device__ __forceinline__ void wait_vm_k() {
    static_assert(N >= 0 && N < 64, "vmcnt range");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ float act_apply(float v, int act, float slope) {
    if (act == VD_ACT_RELU) return v > 0.f ? v : 0.f;
    if (act == VD_ACT_LEAKY) return v > 0.f ? v : v * slope;
    if (act == VD_ACT_SILU) return v / (1.0f + __expf(-v));
    return v;
}

// x = hi + mid + lo exactly (truncation split: each term keeps 8 significand bits)
__device__ __forceinline__ void split3(float x, unsigned& h, unsigned& m, unsigned& l) {
    const unsigned u = __float_as_uint(x);
    const float x0 = __uint_as_float(u & 0xFFFF0000u);
    const float r1 = x - x0;                       // exact
    const unsigned v = __float_as_uint(r1);
    const float x1 = __uint_as_float(v & 0xFFFF0000u);
    const float r2 = r1 - x1;                      // exact, <= 8 significand bits
    h = u >> 16;
    m = v >> 16;
    l = __float_as_uint(r2) >> 16;
}

// x = hi + lo (+ below 2^-24 |x|) with both terms fp16, round to nearest: the
// scaled operand (|x| < 2^15, see act_scale) keeps 22-24 significand bits
__device__ __forceinline__ void split2h(float x, float sa, unsigned& h, unsigned& l) {
    // x * sa is exact (a power of two), so each term is ONE rounding of a fused
    // multiply-add to fp16 (v_fma_mixlo_f16): hi = RNE(x sa), lo = RNE(x sa - hi)
    const _Float16 x0 = (_Float16)__builtin_fmaf(x, sa, 0.f);
    const _Float16 x1 = (_Float16)__builtin_fmaf(x, sa, -(float)x0);   // the residual is exact in f32
    h = __builtin_bit_cast(unsigned short, x0);
    l = __builtin_bit_cast(unsigned short, x1);
}

template <int TERMS>
__device__ __forceinline__ f32x4_t mfma_terms(const u32x4 (&a)[3], const u32x4 (&b)[3], f32x4_t acc);

template <>
__device__ __forceinline__ f32x4_t mfma_terms<3>(const u32x4 (&a)[3], const u32x4 (&b)[3], f32x4_t acc) {
#define VDX_MFMA(pa, pb)                                                                                 \
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a[pa]),                  \
                                                  __builtin_bit_cast(bf16x8_t, b[pb]), acc, 0, 0, 0)
    // small terms first
    VDX_MFMA(2, 0);
    VDX_MFMA(1, 1);
    VDX_MFMA(0, 2);
    VDX_MFMA(1, 0);
    VDX_MFMA(0, 1);
    VDX_MFMA(0, 0);
#undef VDX_MFMA
    return acc;
}

template <>
__device__ __forceinline__ f32x4_t mfma_terms<1>(const u32x4 (&a)[3], const u32x4 (&b)[3], f32x4_t acc) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8_t, a[0]), __builtin_bit_cast(f16x8_t, b[1]),
                                                 acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8_t, a[0]), __builtin_bit_cast(f16x8_t, b[0]),
                                                 acc, 0, 0, 0);
    return acc;
}

template <>
__device__ __forceinline__ f32x4_t mfma_terms<2>(const u32x4 (&a)[3], const u32x4 (&b)[3], f32x4_t acc) {
#define VDH_MFMA(pa, pb)                                                                                 \
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8_t, a[pa]),                    \
                                                 __builtin_bit_cast(f16x8_t, b[pb]), acc, 0, 0, 0)
    VDH_MFMA(1, 0);
    VDH_MFMA(0, 1);
    VDH_MFMA(0, 0);
#undef VDH_MFMA
    return acc;
}

// The same three products in the same order with the operands exchanged: the MFMA
// computes D^T (rows = weight rows / output channels, columns = pixels), so a lane's
// accumulator holds 4 consecutive channels of one pixel (register epilogue, TR tiles)
__device__ __forceinline__ f32x4_t mfma_pair_tr(const u32x4 (&a)[3], const u32x4 (&b)[3], f32x4_t acc) {
#define VDT_MFMA(pa, pb)                                                                                 \
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8_t, b[pb]),                    \
                                                 __builtin_bit_cast(f16x8_t, a[pa]), acc, 0, 0, 0)
    VDT_MFMA(1, 0);
    VDT_MFMA(0, 1);
    VDT_MFMA(0, 0);
#undef VDT_MFMA
    return acc;
}

typedef float f32x16_t __attribute__((ext_vector_type(16)));

// fp16 pair on the 32x32x16 matrix-core form: the same three products per K step of
// 16, half the MFMA instructions of the 16x16x32 form for the same work, and 24 of
// every 32 issue cycles free for the A split / address VALU (16x16x32: 8 of 16)
__device__ __forceinline__ f32x16_t mfma_pair32(const u32x4 (&a)[3], const u32x4 (&b)[3], f32x16_t acc) {
#define VDH_MFMA32(pa, pb)                                                                               \
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8_t, a[pa]),                    \
                                                 __builtin_bit_cast(f16x8_t, b[pb]), acc, 0, 0, 0)
    VDH_MFMA32(1, 0);
    VDH_MFMA32(0, 1);
    VDH_MFMA32(0, 0);
#undef VDH_MFMA32
    return acc;
}

typedef _Float16 half2_t __attribute__((ext_vector_type(2)));

// 8 f32 -> the scaled fp16 pair as two packed 16-B planes, element pairs built in
// half2 registers (v_fma_mixlo / v_fma_mixhi write the halves in place: no shifts or
// ORs); the same roundings as split2h
__device__ __forceinline__ void split_pair8(const float (&e)[8], float sa, u32x4& H, u32x4& L) {
    unsigned hv[4], lv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        half2_t h, l;
        h[0] = (_Float16)__builtin_fmaf(e[2 * j], sa, 0.f);
        h[1] = (_Float16)__builtin_fmaf(e[2 * j + 1], sa, 0.f);
        l[0] = (_Float16)__builtin_fmaf(e[2 * j], sa, -(float)h[0]);
        l[1] = (_Float16)__builtin_fmaf(e[2 * j + 1], sa, -(float)h[1]);
        hv[j] = __builtin_bit_cast(unsigned, h);
        lv[j] = __builtin_bit_cast(unsigned, l);
    }
    H = u32x4{hv[0], hv[1], hv[2], hv[3]};
    L = u32x4{lv[0], lv[1], lv[2], lv[3]};
}

// 8 f32 -> TERMS packed 16-B planes (bf16 truncation split, or scaled fp16 pair)
template <int TERMS>
__device__ __forceinline__ void split_pack(const float (&e)[8], float sa, u32x4 (&o)[3]) {
    if constexpr (TERMS == 2) {
        split_pair8(e, sa, o[0], o[1]);
        return;
    }
    unsigned hv[8], mv[8], lv[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        if constexpr (TERMS == 3) split3(e[j], hv[j], mv[j], lv[j]);
        else if constexpr (TERMS == 2) { split2h(e[j], sa, hv[j], mv[j]); lv[j] = 0; }
        else { hv[j] = __builtin_bit_cast(unsigned short, (_Float16)__builtin_fmaf(e[j], sa, 0.f)); mv[j] = lv[j] = 0; }
    }
    o[0] = u32x4{hv[0] | (hv[1] << 16), hv[2] | (hv[3] << 16), hv[4] | (hv[5] << 16), hv[6] | (hv[7] << 16)};
    if constexpr (TERMS >= 2)
        o[1] = u32x4{mv[0] | (mv[1] << 16), mv[2] | (mv[3] << 16), mv[4] | (mv[5] << 16), mv[6] | (mv[7] << 16)};
    if constexpr (TERMS == 3)
        o[2] = u32x4{lv[0] | (lv[1] << 16), lv[2] | (lv[3] << 16), lv[4] | (lv[5] << 16), lv[6] | (lv[7] << 16)};
}

// The fused epilogue of the 256 / 128-row tiles: BM / EPR passes of EPR accumulator
// rows through LDS, then BN + residual (incl. the FPN nearest-2x source) +
// activation + 16-B stores + the per-frame max |y| into the output's slots.
template <class S, int MF, class AccT>
__device__ __forceinline__ void x6_epilogue(const ConvArgs& a, AccT (&acc)[S::TM][S::TN], int m0, int n0, int wm,
                                            int wn, int tid, int lane, char* smem, int amax_off) {
    constexpr int BM = S::BM, BN = S::BNV, NT = S::NT, TM = S::TM, TN = S::TN, TERMS = S::TERMSV;
    const int ohw = a.yh * a.yw;
    if (a.dbg & 1) {                                   // timing experiment: main loop only
        if (acc[0][0][0] == 1234.5f) ((float*)a.y)[tid] = 1.f;
        return;
    }
    // ---- fused epilogue: BM / EPR passes of EPR rows through LDS ([EPR][BN+4] f32)
    constexpr int EPLD = S::EPLD, EPR = S::EPR, CG = BN / 8, ITEMS = EPR * CG / NT;
    static_assert(ITEMS >= 1 && (EPR * CG) % NT == 0, "epilogue items");
    float* ep = (float*)smem;
    const bool vec_ok = ((a.cout & 7) == 0) && ((a.ldy & 7) == 0) && ((a.ycoff & 7) == 0) &&
                        (a.res_mode == VD_RES_NONE || (((a.res_ld | a.res_coff) & 7) == 0));
    unsigned* s_amax = (unsigned*)(smem + amax_off);   // per-frame max |y| of this tile (a.ymax)
    int tfb = -1;                                      // this thread's first frame and its running max;
    float tmax = 0.f;                                  // items of a later frame go to LDS directly (rare)
#pragma unroll
    for (int h = 0; h < BM / EPR; ++h) {
        if (h) __syncthreads();
        const int wrow = wm * S::WTM - h * EPR;        // this wave's first row within the pass
        if (wrow >= 0 && wrow < EPR) {
            if constexpr (MF == 32) {   // 32x32 C layout: row 8 (r / 4) + 4 (l / 32) + r % 4, column l % 32
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j)
#pragma unroll
                        for (int r = 0; r < 16; ++r)
                            ep[(wrow + i * 32 + 8 * (r >> 2) + 4 * (lane >> 5) + (r & 3)) * EPLD + wn * S::WTN +
                               j * 32 + (lane & 31)] = acc[i][j][r];
            } else {
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j)
#pragma unroll
                        for (int r = 0; r < 4; ++r)
                            ep[(wrow + i * 16 + (lane >> 4) * 4 + r) * EPLD + wn * S::WTN + j * 16 + (lane & 15)] =
                                acc[i][j][r];
            }
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < ITEMS; ++q) {              // EPR rows x CG groups of 8 channels / NT threads
            const int it = tid + NT * q;
            const int rr = it / CG, cg = it % CG;
            const int m = m0 + h * EPR + rr;
            const int nb = n0 + cg * 8;
            const bool valid = m < a.M && nb < a.cout;
            const int fb = valid ? m / ohw : -1;
            float vmax = 0.f;
            if (valid) {
            const float* er = ep + rr * EPLD + cg * 8;
            const size_t yo = (size_t)m * a.ldy + a.ycoff + nb;
            const float inv_sa = TERMS != 3 ? __builtin_ldexpf(1.f, -act_scale_exp(a, fb)) : 1.f;
            size_t roff = 0;
            if (a.res_mode != VD_RES_NONE) {
                if (a.res_up) {
                    const int b = m / ohw, rem = m - b * ohw;
                    const int oy = rem / a.yw, ox = rem - oy * a.yw;
                    roff = ((size_t)(b * a.rh + (oy >> 1)) * a.rw + (ox >> 1)) * a.res_ld + a.res_coff + nb;
                } else {
                    roff = (size_t)m * a.res_ld + a.res_coff + nb;
                }
            }
            if (vec_ok) {
                const float4 s0 = *(const float4*)(a.scale + nb), s1 = *(const float4*)(a.scale + nb + 4);
                const float4 h0 = *(const float4*)(a.shift + nb), h1 = *(const float4*)(a.shift + nb + 4);
                const float sc[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
                const float sh[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
                const float4 e0 = *(const float4*)er, e1 = *(const float4*)(er + 4);
                const float ev[8] = {e0.x, e0.y, e0.z, e0.w, e1.x, e1.y, e1.z, e1.w};
                float rv[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
                if (a.res_mode != VD_RES_NONE) {
                    const float4 r0 = *(const float4*)((const float*)a.res + roff);
                    const float4 r1 = *(const float4*)((const float*)a.res + roff + 4);
                    rv[0] = r0.x; rv[1] = r0.y; rv[2] = r0.z; rv[3] = r0.w;
                    rv[4] = r1.x; rv[5] = r1.y; rv[6] = r1.z; rv[7] = r1.w;
                }
                float v[8];
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    float t = (ev[e] * inv_sa) * sc[e] + sh[e];
                    if (a.res_mode == VD_RES_PRE_ACT) t += rv[e];
                    t = act_apply(t, a.act, a.slope);
                    if (a.res_mode == VD_RES_POST_ACT) t += rv[e];
                    v[e] = t;
                    vmax = fmaxf(vmax, fabsf(t));
                }
                *(float4*)((float*)a.y + yo) = make_float4(v[0], v[1], v[2], v[3]);
                *(float4*)((float*)a.y + yo + 4) = make_float4(v[4], v[5], v[6], v[7]);
            } else {
                for (int e = 0; e < 8 && nb + e < a.cout; ++e) {
                    const int n = nb + e;
                    float t = (er[e] * inv_sa) * a.scale[n] + a.shift[n];
                    const float rv = a.res_mode != VD_RES_NONE ? ((const float*)a.res)[roff + e] : 0.f;
                    if (a.res_mode == VD_RES_PRE_ACT) t += rv;
                    t = act_apply(t, a.act, a.slope);
                    if (a.res_mode == VD_RES_POST_ACT) t += rv;
                    ((float*)a.y)[yo + e] = t;
                    vmax = fmaxf(vmax, fabsf(t));
                }
            }
            }   // valid
            if (valid && a.ymax) {
                if (tfb < 0) tfb = fb;
                if (fb == tfb) tmax = fmaxf(tmax, vmax);
                else if (vmax > 0.f) atomicMax(s_amax + fb, __float_as_uint(vmax));
            }
        }
    }
    if (a.ymax) {
        amax_lds_add(s_amax, tfb, tmax);
        __syncthreads();
        amax_lds_flush(s_amax, a.ymax, a.B);
    }
}

// Epilogue of the transposed (TR) tiles straight from registers: the weight rows were
// loaded permuted (x6_tr_row), so MFMA blocks 2jp, 2jp+1 give lane (p = l % 16, q = l / 16)
// the 8 consecutive channels 32 jp + 8 q .. +7 of pixel 16 i + p: BN + residual +
// activation on 8 values, two 16-B stores, no LDS staging and no workgroup barrier
// (only the per-frame max goes through LDS). Same arithmetic as x6_epilogue.
template <class S>
__device__ __forceinline__ void x6_epilogue_tr(const ConvArgs& a, f32x4_t (&acc)[S::TM][S::TN], int m0, int n0,
                                               int wm, int wn, int lane, unsigned* s_amax) {
    constexpr int TM = S::TM, TN = S::TN, NJ = TN / 2;
    static_assert(TN % 2 == 0, "TR tiles pair the channel blocks");
    const int ohw = a.yh * a.yw;
    const int q = lane >> 4, pl = lane & 15;
    const int cb = n0 + wn * S::WTN + 8 * q;
    int fbs[TM];
    unsigned yrow[TM], rrow[TM];                     // byte offsets of the lane's output / residual row (channel 0)
    float inv[TM], vmax[TM];
    const bool res = a.res_mode != VD_RES_NONE;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
        const int m = m0 + wm * S::WTM + 16 * i + pl;
        const bool ok = m < a.M;
        fbs[i] = ok ? m / ohw : -1;
        inv[i] = __builtin_ldexpf(1.f, -act_scale_exp(a, ok ? fbs[i] : 0));
        vmax[i] = 0.f;
        yrow[i] = ok ? (unsigned)(((size_t)m * a.ldy + a.ycoff) * 4) : 0x80000000u;
        rrow[i] = 0x80000000u;
        if (ok && res) {
            size_t roff;
            if (a.res_up) {
                const int b = fbs[i], rem = m - b * ohw;
                const int oy = rem / a.yw, ox = rem - oy * a.yw;
                roff = ((size_t)(b * a.rh + (oy >> 1)) * a.rw + (ox >> 1)) * a.res_ld;
            } else {
                roff = (size_t)m * a.res_ld;
            }
            rrow[i] = (unsigned)((roff + a.res_coff) * 4);
        }
    }
    // Buffer loads / stores (rows past M, channels past cout: out of range -> zeros /
    // dropped) keep the epilogue straight-line, and column pair jp + 1's residual and
    // BN rows are loaded before pair jp's stores: vmcnt retires loads and stores in issue
    // order, so a residual load issued after a store waited for that store too (the
    // round-5 epilogue waited on every (jp, i) row behind the stores before it).
    const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc(a.y, 0, 0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc((void*)a.res, 0, res ? 0x7fffffff : 0,
                                                                         0x00020000);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)a.scale, 0, a.cout * 4, 0x00020000);
    const __amdgpu_buffer_rsrc_t rh = __builtin_amdgcn_make_buffer_rsrc((void*)a.shift, 0, a.cout * 4, 0x00020000);
    u32x4 rq[2][TM][2], sq[2][4];
    auto fetch = [&](int jp, int slot) {
        const unsigned cbytes = (unsigned)((cb + 32 * jp) * 4);
        sq[slot][0] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)cbytes, 0, 0));
        sq[slot][1] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)cbytes, 16, 0));
        sq[slot][2] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rh, (int)cbytes, 0, 0));
        sq[slot][3] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rh, (int)cbytes, 16, 0));
        if (res) {
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                const unsigned o = rrow[i] == 0x80000000u ? rrow[i] : rrow[i] + cbytes;
                rq[slot][i][0] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rr, (int)o, 0, 0));
                rq[slot][i][1] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rr, (int)o, 16, 0));
            }
        }
    };
    fetch(0, 0);
#pragma unroll
    for (int jp = 0; jp < NJ; ++jp) {
        if (jp + 1 < NJ) fetch(jp + 1, (jp + 1) & 1);
        const int sl = jp & 1;
        const bool cok = cb + 32 * jp < a.cout;
        const unsigned cbytes = (unsigned)((cb + 32 * jp) * 4);
#pragma unroll
        for (int i = 0; i < TM; ++i) {
            float v[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const float ev = e < 4 ? acc[i][2 * jp][e] : acc[i][2 * jp + 1][e - 4];
                const float sc = __uint_as_float(sq[sl][e >> 2][e & 3]), sh = __uint_as_float(sq[sl][2 + (e >> 2)][e & 3]);
                const float rv = res ? __uint_as_float(rq[sl][i][e >> 2][e & 3]) : 0.f;
                float t = (ev * inv[i]) * sc + sh;
                if (a.res_mode == VD_RES_PRE_ACT) t += rv;
                t = act_apply(t, a.act, a.slope);
                if (a.res_mode == VD_RES_POST_ACT) t += rv;
                v[e] = t;
                if (cok && fbs[i] >= 0) vmax[i] = fmaxf(vmax[i], fabsf(t));
            }
            const unsigned o = (yrow[i] == 0x80000000u || !cok) ? 0x80000000u : yrow[i] + cbytes;
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned,
                                                                      make_float4(v[0], v[1], v[2], v[3])),
                                                   ry, (int)o, 0, 0);
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned,
                                                                      make_float4(v[4], v[5], v[6], v[7])),
                                                   ry, (int)o, 16, 0);
        }
    }
    if (a.ymax) {
#pragma unroll
        for (int i = 0; i < TM; ++i) amax_lds_add(s_amax, fbs[i], vmax[i]);
        __syncthreads();
        amax_lds_flush(s_amax, a.ymax, a.B);
    }
}

// the round-5 form (option x6_tr_epi = 0): residual and BN rows loaded row by row behind the stores
template <class S>
__device__ __forceinline__ void x6_epilogue_tr_r5(const ConvArgs& a, f32x4_t (&acc)[S::TM][S::TN], int m0, int n0,
                                               int wm, int wn, int lane, unsigned* s_amax) {
    constexpr int TM = S::TM, TN = S::TN;
    static_assert(TN % 2 == 0, "TR tiles pair the channel blocks");
    const int ohw = a.yh * a.yw;
    const int q = lane >> 4, pl = lane & 15;
    const int cb = n0 + wn * S::WTN + 8 * q;
    int mrow[TM], fbs[TM];
    float inv[TM], vmax[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
        const int m = m0 + wm * S::WTM + 16 * i + pl;
        mrow[i] = m;
        fbs[i] = m < a.M ? m / ohw : -1;
        inv[i] = __builtin_ldexpf(1.f, -act_scale_exp(a, fbs[i] < 0 ? 0 : fbs[i]));
        vmax[i] = 0.f;
    }
#pragma unroll
    for (int jp = 0; jp < TN / 2; ++jp) {
        const int c = cb + 32 * jp;
        if (c >= a.cout) continue;
        const float4 s0 = *(const float4*)(a.scale + c), s1 = *(const float4*)(a.scale + c + 4);
        const float4 h0 = *(const float4*)(a.shift + c), h1 = *(const float4*)(a.shift + c + 4);
        const float sc[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
        const float sh[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
#pragma unroll
        for (int i = 0; i < TM; ++i) {
            const int m = mrow[i];
            if (m >= a.M) continue;
            float rv[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
            if (a.res_mode != VD_RES_NONE) {
                size_t roff;
                if (a.res_up) {
                    const int b = fbs[i], rem = m - b * ohw;
                    const int oy = rem / a.yw, ox = rem - oy * a.yw;
                    roff = ((size_t)(b * a.rh + (oy >> 1)) * a.rw + (ox >> 1)) * a.res_ld;
                } else {
                    roff = (size_t)m * a.res_ld;
                }
                roff += a.res_coff + c;
                const float4 r0 = *(const float4*)((const float*)a.res + roff);
                const float4 r1 = *(const float4*)((const float*)a.res + roff + 4);
                rv[0] = r0.x; rv[1] = r0.y; rv[2] = r0.z; rv[3] = r0.w;
                rv[4] = r1.x; rv[5] = r1.y; rv[6] = r1.z; rv[7] = r1.w;
            }
            float v[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const float ev = e < 4 ? acc[i][2 * jp][e] : acc[i][2 * jp + 1][e - 4];
                float t = (ev * inv[i]) * sc[e] + sh[e];
                if (a.res_mode == VD_RES_PRE_ACT) t += rv[e];
                t = act_apply(t, a.act, a.slope);
                if (a.res_mode == VD_RES_POST_ACT) t += rv[e];
                v[e] = t;
                vmax[i] = fmaxf(vmax[i], fabsf(t));
            }
            float* yp = (float*)a.y + (size_t)m * a.ldy + a.ycoff + c;
            *(float4*)yp = make_float4(v[0], v[1], v[2], v[3]);
            *(float4*)(yp + 4) = make_float4(v[4], v[5], v[6], v[7]);
        }
    }
    if (a.ymax) {
#pragma unroll
        for (int i = 0; i < TM; ++i) amax_lds_add(s_amax, fbs[i], vmax[i]);
        __syncthreads();
        amax_lds_flush(s_amax, a.ymax, a.B);
    }
}

// LDS row -> weight row of a TR tile: row 16 j + i of each 32-row group holds channel
// 8 (i >> 2) + 4 (j & 1) + (i & 3) of the group, so blocks 2jp, 2jp+1 give a lane 8
// consecutive channels (conv1x1_x6_kernel's permutation)
// the register epilogue (x6_epilogue_tr) addresses y and the residual by 32-bit buffer offsets
static bool tr_bytes_ok(const ConvArgs& a) {
    const double lim = 2147483647.0;
    if ((double)a.M * a.ldy * 4 >= lim) return false;
    if (a.res_mode != VD_RES_NONE && (double)a.M * a.res_ld * 4 >= lim) return false;
    return true;
}

__device__ __forceinline__ int x6_tr_row(int row) {
    const int j = (row >> 4) & 1, i = row & 15;
    return (row & ~31) + 8 * (i >> 2) + 4 * j + (i & 3);
}

template <int BM, int BN, int NT, int NST, int TERMS, int MF, int NA, bool TR = false, bool PF = false>
// NA: A register sets (K tiles of A loads in flight: NA - 1 besides the one being split)
// 8 waves: two workgroups' worth of waves per SIMD pair (256 VGPRs each); 4 waves (one
// per SIMD, 128 x 128 wave tiles): the whole 512-register file per wave, the
// accumulators in AGPRs
// TR: transposed accumulators (D^T, weight rows permuted by x6_tr_row) and the register
// epilogue x6_epilogue_tr; fp16 pairs on the 16x16x32 form only
__global__ __launch_bounds__(NT, NT == 256 && BM == 256 ? 1 : 2) void conv_x6_kernel(ConvArgs a) {
    static_assert(MF == 16 || (MF == 32 && TERMS == 2), "32x32x16 form: fp16 pairs only");
    static_assert(!TR || (MF == 16 && TERMS == 2), "TR tiles: fp16 pairs on 16x16x32");
    using S = X6Shape<BM, BN, NT, NST, TERMS, MF>;
    constexpr int STAGE = S::STAGE, PL_A = S::PL_A, PL_B = S::PL_B, TM = S::TM, TN = S::TN, WAVES = S::WAVES;
    constexpr int AROWS = S::AROWS, AIT = S::AITEMS;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid / S::WAVES_N, wn = wid % S::WAVES_N;

    // XCD-aware bijective remap (blocks b, b+8, ... share an XCD)
    const int nwg = gridDim.x, bid = blockIdx.x;
    const int q8 = nwg >> 3, r8 = nwg & 7, xcd = bid & 7;
    const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
    const int tn = wg % a.ntiles_n, tm = wg / a.ntiles_n;
    const int m0 = a.mbase + tm * BM, n0 = tn * BN;

    // ---- A staging: thread = (row, k-pair) items; item i: row = (tid >> 2) + AROWS i, pair = tid & 3 (k 8p..8p+7)
    const int apair = tid & 3, arow = tid >> 2;
    const int ohw = a.yh * a.yw;
    int pix0[AIT];                                  // element offsets (xbytes < 2^31: vd_conv_x6_ok)
    int iy0[AIT], ix0[AIT];
    float sa[AIT];                                  // fp16 pair: the row's frame scale 2^k
#pragma unroll
    for (int i = 0; i < AIT; ++i) {
        sa[i] = 1.f;
        const int m = m0 + arow + AROWS * i;
        if (m < a.M) {
            const int b = m / ohw, rem = m - b * ohw;
            const int oy = rem / a.yw, ox = rem - oy * a.yw;
            iy0[i] = oy * a.stride - a.pad;
            ix0[i] = ox * a.stride - a.pad;
            pix0[i] = ((b * a.xh + iy0[i]) * a.xw + ix0[i]) * a.ldx + a.xcoff;
            if constexpr (TERMS != 3) sa[i] = __builtin_ldexpf(1.f, act_scale_exp(a, b));
        } else {
            iy0[i] = -(1 << 28); ix0[i] = 0; pix0[i] = 0;
        }
    }
    const int tap_dy = a.xw * a.ldx;
    const int nk = a.kpad / KT;
    // A through a buffer descriptor: 32-bit byte offsets, and an offset past
    // num_records returns zeros (conv padding, K padding) without a select on the
    // loaded value -- a select would force a wait right at the load
    const long xbytes = (long)a.B * a.xh * a.xw * a.ldx * 4;
    const __amdgpu_buffer_rsrc_t rsrc_x = __builtin_amdgcn_make_buffer_rsrc((void*)a.x, 0, (int)xbytes, 0x00020000);
    // 1x1 convs without K padding (option x6_one): K tile kt of a row is bytes
    // [128 kt, 128 kt + 128) past the row's pixel, so each load is the row's byte offset
    // (rows past M: out of range) plus a scalar offset -- no per-tile tap stepping
    const bool one = (a.dbg & 4) && a.kh == 1 && a.kw == 1 && a.pad == 0 &&
                     a.kpad == a.cin_pad && a.cin_pad % KT == 0;
    if (one) {
#pragma unroll
        for (int i = 0; i < AIT; ++i)
            pix0[i] = m0 + arow + AROWS * i < a.M ? pix0[i] * 4 + apair * 32 : (int)0x80000000;
    }
    int lk = 0;                                     // K tiles loaded so far (one: the scalar offset)
    // The two-stage main loop on 1x1 convs (UNI) issues the same loads and DMAs every
    // iteration (past nk: the last tile again, L2 hits), branch-free, so that the
    // compiler's own waits on the A registers count every younger op -- with the refills
    // under `if`s (and the runtime `one` branch) it assumed none and waited for the NEXT
    // tile's loads (just issued) in the middle of the MFMAs

    // two register sets of A (8 f32 of each of 2 rows): tile t lives in set t & 1,
    // loaded two iterations before it is split into LDS
    u32x4 ra[NA][AIT][2];                           // [set][item][half]
    // per half h: the (dy, dx, c) of this thread's 4-channel chunk kt*8 + 2*apair + h,
    // advanced by 32 channels per load_a call (tiles are loaded in order): no
    // divisions and no branches in the load path
    int tdy[2], tdx[2], tc[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int ch0 = (apair * 2 + h) * 4;
        const int t = ch0 / a.cin_pad;
        tc[h] = ch0 - t * a.cin_pad;
        tdy[h] = t / a.kw;
        tdx[h] = t - tdy[h] * a.kw;
    }
    auto load_a_any = [&](u32x4 (&r)[AIT][2]) {
        if (one) {
            const int so = lk * (KT * 4);
#pragma unroll
            for (int i = 0; i < AIT; ++i) {
                r[i][0] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rsrc_x, pix0[i], so, 0));
                r[i][1] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rsrc_x, pix0[i] + 16, so, 0));
            }
            ++lk;
            return;
        }
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            // a chunk past the last tap (K padding) is pushed off the image rows, so
            // one unsigned compare rejects it (selects only: no divergent branch)
            const int dyk = tdy[h] < a.kh ? tdy[h] : (1 << 28);
            const int toff = tdy[h] * tap_dy + tdx[h] * a.ldx + tc[h];
#pragma unroll
            for (int i = 0; i < AIT; ++i) {
                const unsigned iy = (unsigned)(iy0[i] + dyk), ix = (unsigned)(ix0[i] + tdx[h]);
                const bool ok = (iy < (unsigned)a.xh) & (ix < (unsigned)a.xw);
                const unsigned off = ok ? (unsigned)(pix0[i] + toff) * 4u : 0x80000000u;
                r[i][h] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rsrc_x, (int)off, 0, 0));
            }
            tc[h] += KT;
            if (a.cin_pad >= KT) {                  // at most one tap step per tile: selects only
                const bool wrap = tc[h] >= a.cin_pad;
                tc[h] -= wrap ? a.cin_pad : 0;
                tdx[h] += wrap ? 1 : 0;
                const bool wrap2 = tdx[h] >= a.kw;
                tdx[h] -= wrap2 ? a.kw : 0;
                tdy[h] += wrap2 ? 1 : 0;
            } else {
                while (tc[h] >= a.cin_pad) { tc[h] -= a.cin_pad; ++tdx[h]; }
                while (tdx[h] >= a.kw) { tdx[h] -= a.kw; ++tdy[h]; }
            }
        }
    };
    auto store_item = [&](int st, const u32x4 (&r)[AIT][2], int i) {
        char* A = smem + st * STAGE;
        float e[8];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            e[j] = __uint_as_float(r[i][0][j]);
            e[4 + j] = __uint_as_float(r[i][1][j]);
        }
        u32x4 o[3];
        split_pack<TERMS>(e, sa[i], o);
        const int off = swz(arow + AROWS * i, apair);
#pragma unroll
        for (int p = 0; p < S::TA; ++p) *(u32x4*)(A + p * PL_A + off) = o[p];
    };

    // ---- B: LDS-DMA, one instruction = 1 KB = 16 rows of one plane; NDMA per tile,
    // instruction j on wave j % WAVES: plane j / (BN/16), rows 16 * (j % (BN/16)) .. +15
    constexpr int RB = BN / 16;                        // 16-row blocks per plane
    constexpr int NDMA = S::NDMA;
    const int my_dma = NDMA / WAVES + (wid < NDMA % WAVES ? 1 : 0);
    const __amdgpu_buffer_rsrc_t rsrc_w = __builtin_amdgcn_make_buffer_rsrc((void*)a.w, 0, 0x7fffffff, 0x00020000);
    auto dma_b = [&](int kt, int st) {
        char* Bs = smem + st * STAGE + S::TA * PL_A;
#pragma unroll
        for (int q = 0; q < (NDMA + WAVES - 1) / WAVES; ++q) {
            const int j = wid + WAVES * q;
            if (NDMA % WAVES == 0 || j < NDMA) {
                const int p = j / RB, r0 = (j % RB) * 16;
                const int row = r0 + (lane >> 2), slot = lane & 3;
                const int chunk = slot ^ (((row >> 3) & 1) * 3);
                const int wrow = TR ? x6_tr_row(row) : row;
                const int ktc = kt < nk ? kt : nk - 1;     // UNI tail: the last tile again (a scalar min)
                const unsigned off = (unsigned)((((long)(n0 + wrow) * nk + ktc) * S::TB + p) * 64 + chunk * 16);
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc_w, (lds_void_t*)(Bs + p * PL_B + r0 * 64), 16, off, 0,
                                                         0, 0);
            }
        }
    };

    using AccT = typename std::conditional<MF == 32, f32x16_t, f32x4_t>::type;
    AccT acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = AccT{};
    if (a.ymax)   // beyond the stages / epilogue image; ordered before use by the main loop's barriers
        for (int f = tid; f < a.B; f += NT) ((unsigned*)(smem + S::LDS))[f] = 0u;

    // one K tile from stage st; the split + LDS write of the next tile's A items are
    // interleaved with the MFMA rows (VALU work beside the matrix cores)
    auto compute = [&](int st, bool split_next, int st_next, const u32x4 (&rn)[AIT][2]) {
        const char* A = smem + st * STAGE;
        const char* Bs = A + S::TA * PL_A;
        const int ch = lane >> 4;
        if constexpr (MF == 32) {   // two K steps of 16: lane l reads row l % 32, 16-B chunk 2 s + l / 32
            const int r32 = lane & 31, c32 = lane >> 5;
#pragma unroll
            for (int sk = 0; sk < 2; ++sk) {
                u32x4 af[TM][3];
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int p = 0; p < 2; ++p)
                        af[i][p] = *(const u32x4*)(A + p * PL_A + swz(wm * S::WTM + i * 32 + r32, 2 * sk + c32));
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    u32x4 bf[3];
#pragma unroll
                    for (int p = 0; p < 2; ++p)
                        bf[p] = *(const u32x4*)(Bs + p * PL_B + swz(wn * S::WTN + j * 32 + r32, 2 * sk + c32));
#pragma unroll
                    for (int i = 0; i < TM; ++i) acc[i][j] = mfma_pair32(af[i], bf, acc[i][j]);
#pragma unroll
                    for (int q = 0; q < AIT; ++q)
                        if (split_next && sk == q * 2 / AIT && j == (q * 2 % AIT) * TN / AIT) store_item(st_next, rn, q);
                }
            }
        } else if constexpr (TN > TM && PF) {
            // PF (option x6_gemm_pf): B fragments of column block j + 1 read before the MFMAs
            // of block j (two buffers), pinned by scheduling groups (as the halo tiles)
            u32x4 af[TM][3], bq[2][3];
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int p = 0; p < S::TA; ++p)
                    af[i][p] = *(const u32x4*)(A + p * PL_A + swz(wm * S::WTM + i * 16 + (lane & 15), ch));
#pragma unroll
            for (int p = 0; p < S::TB; ++p) bq[0][p] = *(const u32x4*)(Bs + p * PL_B + swz(wn * S::WTN + (lane & 15), ch));
            __builtin_amdgcn_sched_group_barrier(0x0100, TM * S::TA + S::TB, 0);
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                if (j + 1 < TN) {
#pragma unroll
                    for (int p = 0; p < S::TB; ++p)
                        bq[(j + 1) & 1][p] = *(const u32x4*)(Bs + p * PL_B + swz(wn * S::WTN + (j + 1) * 16 + (lane & 15), ch));
                    __builtin_amdgcn_sched_group_barrier(0x0100, S::TB, 0);
                }
#pragma unroll
                for (int i = 0; i < TM; ++i) {
                    if constexpr (TR) acc[i][j] = mfma_pair_tr(af[i], bq[j & 1], acc[i][j]);
                    else acc[i][j] = mfma_terms<TERMS>(af[i], bq[j & 1], acc[i][j]);
                }
                __builtin_amdgcn_sched_group_barrier(0x0008, (TERMS == 3 ? 6 : TERMS == 2 ? 3 : 2) * TM, 0);
#pragma unroll
                for (int q = 0; q < AIT; ++q)
                    if (split_next && j == q * TN / AIT) store_item(st_next, rn, q);
            }
        } else if constexpr (TN > TM) {   // wide wave tile: all A fragments resident, B fragments streamed
            u32x4 af[TM][3];
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int p = 0; p < S::TA; ++p)
                    af[i][p] = *(const u32x4*)(A + p * PL_A + swz(wm * S::WTM + i * 16 + (lane & 15), ch));
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                u32x4 bf[3];
#pragma unroll
                for (int p = 0; p < S::TB; ++p)
                    bf[p] = *(const u32x4*)(Bs + p * PL_B + swz(wn * S::WTN + j * 16 + (lane & 15), ch));
#pragma unroll
                for (int i = 0; i < TM; ++i) {
                    if constexpr (TR) acc[i][j] = mfma_pair_tr(af[i], bf, acc[i][j]);
                    else acc[i][j] = mfma_terms<TERMS>(af[i], bf, acc[i][j]);
                }
#pragma unroll
                for (int q = 0; q < AIT; ++q)
                    if (split_next && j == q * TN / AIT) store_item(st_next, rn, q);
            }
        } else {
            u32x4 bf[TN][3];
#pragma unroll
            for (int j = 0; j < TN; ++j)
#pragma unroll
                for (int p = 0; p < S::TB; ++p)
                    bf[j][p] = *(const u32x4*)(Bs + p * PL_B + swz(wn * S::WTN + j * 16 + (lane & 15), ch));
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                u32x4 af[3];
#pragma unroll
                for (int p = 0; p < S::TA; ++p)
                    af[p] = *(const u32x4*)(A + p * PL_A + swz(wm * S::WTM + i * 16 + (lane & 15), ch));
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    if constexpr (TR) acc[i][j] = mfma_pair_tr(af, bf[j], acc[i][j]);
                    else acc[i][j] = mfma_terms<TERMS>(af, bf[j], acc[i][j]);
                }
                if constexpr (AIT == 2) {
                    if (split_next && i == 0) store_item(st_next, rn, 0);
                    if (split_next && i == (TM > 2 ? 2 : 1)) store_item(st_next, rn, 1);
                } else {
#pragma unroll
                    for (int q = 0; q < AIT; ++q)
                        if (split_next && i == q * TM / AIT) store_item(st_next, rn, q);
                }
            }
        }
    };

    if constexpr (NST == 2) {
    // ---- main loop. A(t) lives in register set t % NA. Per thread VMEM issue order at
    // the end of iteration t: A(t+1+NA) loads (2 AIT, into the set A(t+1) just left),
    // B(t+2) DMA (my_dma); the prologue issues A(0) (split at once), A(1..NA-1), B(0),
    // A(NA), B(1), i.e. the ends of iterations -2 and -1. At the top of iteration t the
    // ops younger than B(t) are those of iteration t-1's end, and A(t+1) is older than
    // B(t), so both retire at vmcnt(2 AIT + my_dma) (fewer when the tail issued less).
    // UNI (default; option x6_gemm_uni 0 = the round-5 loop): every iteration issues its
    // loads and DMA (past nk: out of range), the loop runs whole rounds of NA iterations
    // and a tail after it, so the compiler's waits on the A registers see every younger op
    // ONEB (option x6_gemm_uni 2): one barrier per K tile -- B(kt+1)'s DMA and A(kt+NA)'s
    // loads issued right after tile kt's barrier (stage (kt+1) & 1 was last read by tile
    // kt-1, which every wave has finished there), so the barrier after the MFMAs goes
    auto main_loop = [&](auto mode_tag) {
    constexpr int MODE = decltype(mode_tag)::value;
    constexpr bool UNI = MODE >= 1;
    auto load_a = [&](u32x4 (&r)[AIT][2]) {
        if constexpr (UNI) {                                  // 1x1 (one): no tap stepping, no branch
            const int so = (lk < nk ? lk : nk - 1) * (KT * 4);
#pragma unroll
            for (int i = 0; i < AIT; ++i) {
                r[i][0] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rsrc_x, pix0[i], so, 0));
                r[i][1] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rsrc_x, pix0[i] + 16, so, 0));
            }
            ++lk;
        } else {
            load_a_any(r);
        }
    };
    load_a(ra[0]);
#pragma unroll
    for (int q = 0; q < AIT; ++q) store_item(0, ra[0], q);
    if constexpr (MODE == 2) {
        // VMEM order: A(1..NA-2), B(0), A(NA-1) | per tile kt after its barrier: B(kt+1),
        // A(kt+NA). Younger than B(kt) at the top of kt: A(kt-1+NA) only.
#pragma unroll
        for (int j = 1; j < NA - 1; ++j) load_a(ra[j]);
        dma_b(0, 0);
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("" ::: "memory");
        load_a(ra[NA - 1]);
        auto iterb = [&](int kt, const u32x4 (&rnext)[AIT][2], u32x4 (&rfree)[AIT][2]) {
            wait_vm_k<2 * AIT>();
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // this thread's A(kt) ds_writes
            __builtin_amdgcn_s_barrier();                        // B(kt), A(kt) visible; tile kt-1 done
            asm volatile("" ::: "memory");
            dma_b(kt + 1, (kt + 1) & 1);
            // the wait above counts the A loads as the youngest ops: the scheduler may not
            // interleave them with the DMA (it did, and a DMA left in flight raced the reads)
            __builtin_amdgcn_sched_barrier(0);
            asm volatile("" ::: "memory");
            load_a(rfree);                                       // A(kt+NA) into the set A(kt) left
            compute(kt & 1, kt + 1 < nk, (kt + 1) & 1, rnext);
        };
        int kt = 0;
        for (; kt + NA <= nk; kt += NA) {
#pragma unroll
            for (int u = 0; u < NA; ++u) iterb(kt + u, ra[(u + 1) % NA], ra[u]);
        }
#pragma unroll
        for (int u = 0; u < NA - 1; ++u)
            if (kt + u < nk) iterb(kt + u, ra[(u + 1) % NA], ra[u]);
        wait_vm_k<0>();                                          // the tail's DMA / loads (past nk)
        return;
    }
#pragma unroll
    for (int j = 1; j < NA; ++j)
        if (UNI || j < nk) load_a(ra[j]);
    dma_b(0, 0);
    if (UNI || NA < nk) load_a(ra[0]);
    if (UNI || nk > 1) dma_b(1, 1);
    auto iter = [&](int kt, const u32x4 (&rnext)[AIT][2], u32x4 (&rfree)[AIT][2]) {
        if (S::NDMA % WAVES == 0 && !(a.dbg & 2)) {   // immediates: no runtime wait_vm branch tree
            constexpr int MYD = S::NDMA % WAVES == 0 ? S::NDMA / WAVES : 0;
            if (UNI || kt + NA < nk) wait_vm_k<2 * AIT + MYD>();
            else if (kt + 1 < nk) wait_vm_k<MYD>();
            else wait_vm_k<0>();
        } else {
            wait_vm(UNI ? 2 * AIT + my_dma : (kt + NA < nk ? 2 * AIT : 0) + (kt + 1 < nk ? my_dma : 0));
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // this thread's A(kt) ds_writes
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        compute(kt & 1, kt + 1 < nk, (kt + 1) & 1, rnext);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();                        // everyone done reading stage kt & 1
        asm volatile("" ::: "memory");
        if (UNI || kt + 1 + NA < nk) load_a(rfree);           // A(kt+1+NA) into the set A(kt+1) just left
        if (UNI || kt + 2 < nk) dma_b(kt + 2, kt & 1);
    };
    // Raw barriers with counted waits: __syncthreads() would add vmcnt(0) and drain
    // the prefetch. Unrolled by NA so the register sets are indexed statically.
    if constexpr (UNI) {
        int kt = 0;
        for (; kt + NA <= nk; kt += NA) {
#pragma unroll
            for (int u = 0; u < NA; ++u) iter(kt + u, ra[(u + 1) % NA], ra[(u + 1) % NA]);
        }
#pragma unroll
        for (int u = 0; u < NA - 1; ++u)
            if (kt + u < nk) iter(kt + u, ra[(u + 1) % NA], ra[(u + 1) % NA]);
        wait_vm_k<0>();                                       // the out-of-range tail ops
    } else {
        for (int kt = 0; kt < nk; kt += NA) {
#pragma unroll
            for (int u = 0; u < NA; ++u)
                if (kt + u < nk) iter(kt + u, ra[(u + 1) % NA], ra[(u + 1) % NA]);
        }
    }
    };
    bool looped = false;
    if constexpr (S::NDMA % WAVES == 0) {
        if (one && (a.dbg & 2048)) {
            main_loop(std::integral_constant<int, 2>{});
            looped = true;
        }
    }
    if (!looped) {
        if (one && !(a.dbg & 1024)) main_loop(std::integral_constant<int, 1>{});
        else main_loop(std::integral_constant<int, 0>{});
    }
    } else {
    // ---- one LDS stage: per tile, B(kt) DMA and the split A(kt) write, then
    // compute; A(kt+1)'s loads run under it (registers), B waits for the stage
    load_a_any(ra[0]);
    auto iter1 = [&](int kt, const u32x4 (&rcur)[AIT][2], u32x4 (&rnext)[AIT][2]) {
        dma_b(kt, 0);
#pragma unroll
        for (int q = 0; q < AIT; ++q) store_item(0, rcur, q);   // compiler waits for A(kt)'s loads
        if (kt + 1 < nk) load_a_any(rnext);
        if (kt + 1 < nk) wait_vm_k<2 * AIT>();                // B(kt) landed (older than A(kt+1))
        else wait_vm_k<0>();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        compute(0, false, 0, rcur);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();                        // the stage is free again
        asm volatile("" ::: "memory");
    };
    for (int kt = 0; kt < nk; kt += 2) {
        iter1(kt, ra[0], ra[1]);
        if (kt + 1 < nk) iter1(kt + 1, ra[1], ra[0]);
    }
    }
    if constexpr (TR) {
        if (a.dbg & 1) {                               // timing experiment: main loop only
            if (acc[0][0][0] == 1234.5f) ((float*)a.y)[tid] = 1.f;
            return;
        }
        if (a.dbg & 512) x6_epilogue_tr_r5<S>(a, acc, m0, n0, wm, wn, lane, (unsigned*)(smem + S::LDS));
        else x6_epilogue_tr<S>(a, acc, m0, n0, wm, wn, lane, (unsigned*)(smem + S::LDS));
    } else {
        __syncthreads();
        x6_epilogue<S, MF>(a, acc, m0, n0, wm, wn, tid, lane, smem, S::LDS);
    }
}

// ---------------------------------------------------------------------------
// 3x3 / stride 1 / pad 1 convs on fp16 pairs with the input split ONCE per 32-channel
// chunk (option x6_halo). The 256 output rows of a tile are 256 consecutive pixels
// m0..m0+255 (any frames); tap (dy, dx) of row r reads input pixel m + dy W + dx, so
// all nine taps of a chunk read inside the linear "halo" m0 - W - 1 .. m0 + 256 + W.
// The K loop runs chunk-major (chunk c, then its nine taps): the halo's f32 rows of
// chunk c are loaded once (registers, during chunk c-1's taps), split into fp16
// hi / lo planes once and written to LDS; each tap's A fragments are then halo rows
// shifted by dy W + dx, a padded tap (off the frame's rows or columns, or past M)
// reads a zero row instead -- the per-lane row address carries the padding. The
// conv_x6_kernel path splits every input element nine times (once per tap) and
// loads it nine times; B (the pre-split weights of tap t, chunk c = K tile t CH + c)
// arrives by LDS-DMA into NSB stages: with two, two barriers per K tile as there;
// with three, the stage a DMA refills was last read two tiles ago, so one barrier per
// K tile (plus one per chunk before the halo is rewritten). Same products, same f32
// accumulation, K summed in another order (chunk-major instead of tap-major).
// Halo planes: A fragments start at any row (base + dy W + dx), so the chunk swizzle
// keys on row bit 2 -- conflict-free ds_read_b128 fragment reads (16 rows, two chunks
// per lane group) for every start row, where swz's bit-3 key is conflict-free only
// for starts that are multiples of 8 (checked exhaustively over the 8 start residues)
__device__ __forceinline__ int swzh(int row, int chunk) { return row * 64 + ((chunk ^ (((row >> 2) & 1) << 1)) << 4); }

// TR (round 4, option x6_halo_tr): the MFMA operands exchanged as on the TR GEMM tiles
// (weight rows permuted by x6_tr_row in the DMA, D^T accumulators), so the epilogue runs
// from registers (x6_epilogue_tr) with no LDS staging passes: bit-identical.
//
// S2 (round 5, option x6_halo_s2): 3x3 / stride 2 / pad 1 by phase decomposition. Input
// pixel (2 yo + dy, 2 xo + dx) of output (yo, xo) lies in phase image (py, px) = (dy != 0,
// dx != 0) -- input rows / columns of one parity, an Ho x Wo image indexed like the
// output -- at phase pixel (yo - (dy < 0), xo - (dx < 0)). So each tap reads its phase
// image at a shift of 0 or -1 row / column, the stride-1 halo trick with the halo rows
// m0 - Wo - 1 .. m0 + 255 of one phase image at a time. Per 32-channel chunk the four
// phase halos are split and staged in turn -- phase (1,1) with taps (+-1, +-1), (1,0)
// with (+-1, 0), (0,1) with (0, +-1), (0,0) with (0, 0) -- each loaded into registers
// under the previous phase's taps. A shift-0 tap never crosses a frame (the phase
// pixel is the output pixel's own), a shift of -1 needs yo > 0 / xo > 0, and an odd
// row / column past an odd-sized input is a zero load. conv_x6_kernel splits every
// input element of a stride-2 3x3 conv ~2.25 times per chunk (once per tap that reads
// it); here ~1.3 (the phase halos' overlap). K runs chunk-major in phase order: a
// fixed order for every output (batch invariance), another f32 summation order than
// the tap-major GEMM.
__host__ __device__ __forceinline__ constexpr int s2_tap(int j) {   // step j of a chunk -> weight tap (dy + 1) * 3 + dx + 1
    return j == 0 ? 8 : j == 1 ? 6 : j == 2 ? 2 : j == 3 ? 0 : j == 4 ? 7 : j == 5 ? 1 : j == 6 ? 5 : j == 7 ? 3 : 4;
}
__host__ __device__ __forceinline__ constexpr bool s2_last(int j) { return j == 3 || j == 5 || j == 7 || j == 8; }   // a phase ends

template <int BN, int NSB, bool TR = false, bool S2 = false, bool PF = false>
__global__ __launch_bounds__(512, BN <= 64 ? 4 : 2) void conv_x6_halo_kernel(ConvArgs a) {
    using S = X6Shape<256, BN, 512, 2, 2>;
    constexpr int BM = 256, NT = 512, TM = S::TM, TN = S::TN, WAVES = S::WAVES, PL_B = S::PL_B;
    constexpr int QI = 4;                           // halo items (row, 8 channels) per thread: HR <= 512
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid / S::WAVES_N, wn = wid % S::WAVES_N;
    const int nwg = gridDim.x, bid = blockIdx.x;
    const int q8 = nwg >> 3, r8 = nwg & 7, xcd = bid & 7;
    const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
    const int tn = wg % a.ntiles_n, tm = wg / a.ntiles_n;
    const int m0 = a.mbase + tm * BM, n0 = tn * BN;
    static_assert(!S2 || (NSB == 3 && S::NDMA % WAVES == 0), "stride-2 halo: three B stages, whole DMA rounds");
    const int W = a.yw, H = a.yh, HW = H * W;
    const int HR = S2 ? BM + W + 1 : BM + 2 * W + 2, HP = HR + 1;   // halo rows + one zero row (index HR)
    const int PL_H = HP * 64;
    char* Ah = smem + NSB * 2 * PL_B;               // after the B stages
    const int CH = a.cin_pad / 32, nsteps = 9 * CH, nk = a.kpad / KT;
    const int nhalo = S2 ? 4 * CH : CH;             // halos per tile (S2: four phase images per chunk)

    // ---- halo staging: item i = tid + NT q: row hr = i >> 2, 8 channels pr = i & 3
    const long xbytes = (long)a.B * a.xh * a.xw * a.ldx * 4;
    const __amdgpu_buffer_rsrc_t rsrc_x = __builtin_amdgcn_make_buffer_rsrc((void*)a.x, 0, (int)xbytes, 0x00020000);
    int hoff[QI];                                    // element offset of the item's pixel + channels
    unsigned hexp = 0;                              // the items' frame scale exponents, a byte each
    unsigned hodd = 0;                              // S2: item q's odd input row (bit 2q) / column (2q+1) exists
    const int xg = a.grp_co ? (n0 / a.grp_co) * a.grp_ci : 0;   // grouped conv: this N tile's input group
#pragma unroll
    for (int q = 0; q < QI; ++q) {
        const int it = tid + NT * q, hr = it >> 2, pr = it & 3;
        const int pix = m0 - W - 1 + hr;
        const bool ok = hr < HR && pix >= 0 && pix < a.M;
        if constexpr (S2) {   // phase pixel pix = (b, yo, xo): phase (0, 0) input pixel (b, 2 yo, 2 xo)
            const int b = pix / HW, rem = pix - b * HW, yo = rem / W, xo = rem - yo * W;
            hoff[q] = ok ? ((b * a.xh + 2 * yo) * a.xw + 2 * xo) * a.ldx + a.xcoff + xg + pr * 8 : -1;
            hodd |= (unsigned)((2 * yo + 1 < a.xh ? 1 : 0) | (2 * xo + 1 < a.xw ? 2 : 0)) << (2 * q);
        } else {
            hoff[q] = ok ? pix * a.ldx + a.xcoff + xg + pr * 8 : -1;
        }
        hexp |= (unsigned)((ok ? act_scale_exp(a, pix / HW) : 0) & 0xff) << (8 * q);
    }
    u32x4 hx[QI][2];
    // halo h: chunk h (stride 1); chunk h / 4, phase (py, px) = (1,1) (1,0) (0,1) (0,0) for h % 4 (S2)
    auto load_halo = [&](int h) {
        const int c = S2 ? h >> 2 : h, ph = S2 ? 3 - (h & 3) : 0, py = ph >> 1, px = ph & 1;
        const int dph = (py * a.xw + px) * a.ldx;
        const unsigned need = (unsigned)(py | (px << 1));
#pragma unroll
        for (int q = 0; q < QI; ++q) {
            const bool v = hoff[q] >= 0 && (!S2 || ((hodd >> (2 * q)) & need) == need);
            const unsigned off = v ? (unsigned)(hoff[q] + dph + c * KT) * 4u : 0x80000000u;
            hx[q][0] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rsrc_x, (int)off, 0, 0));
            hx[q][1] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rsrc_x, (int)off, 16, 0));
        }
    };
    auto store_halo = [&]() {
#pragma unroll
        for (int q = 0; q < QI; ++q) {
            const int it = tid + NT * q, hr = it >> 2, pr = it & 3;
            if (hr < HR) {
                float e[8];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    e[j] = __uint_as_float(hx[q][0][j]);
                    e[4 + j] = __uint_as_float(hx[q][1][j]);
                }
                u32x4 o[3];
                const int ex = (int)(signed char)((hexp >> (8 * q)) & 0xff);
                split_pack<2>(e, __builtin_ldexpf(1.f, ex), o);
                *(u32x4*)(Ah + swzh(hr, pr)) = o[0];
                *(u32x4*)(Ah + PL_H + swzh(hr, pr)) = o[1];
            }
        }
    };

    // ---- B: LDS-DMA as conv_x6_kernel, K tile of step s = tap * CH + chunk
    constexpr int RB = BN / 16, NDMA = S::NDMA;
    const int my_dma = NDMA / WAVES + (wid < NDMA % WAVES ? 1 : 0);
    const __amdgpu_buffer_rsrc_t rsrc_w = __builtin_amdgcn_make_buffer_rsrc((void*)a.w, 0, 0x7fffffff, 0x00020000);
    // piece q of this wave's DMA share of step s's K tile into stage st
    auto dma_piece = [&](int s, int st, int q) {
        const int c = s / 9, j = s - 9 * c, kt = (S2 ? s2_tap(j) : j) * CH + c;
        char* Bs = smem + st * 2 * PL_B;
        const int jd = wid + WAVES * q;
        if (jd < NDMA) {
            const int p = jd / RB, r0 = (jd % RB) * 16;
            const int row = r0 + (lane >> 2), slot = lane & 3;
            const int chunk = slot ^ (((row >> 3) & 1) * 3);
            const int wrow = TR ? x6_tr_row(row) : row;
            const unsigned off = (unsigned)((((long)(n0 + wrow) * nk + kt) * 2 + p) * 64 + chunk * 16);
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc_w, (lds_void_t*)(Bs + p * PL_B + r0 * 64), 16, off, 0,
                                                     0, 0);
        }
    };
    auto dma_b = [&](int s, int st) {
#pragma unroll
        for (int q = 0; q < (NDMA + WAVES - 1) / WAVES; ++q) dma_piece(s, st, q);
    };
    // where a step issues the DMA of step s + 2 (option x6_halo_dma, whole DMA rounds only):
    // 0 right after the step's barrier, 1 after its MFMAs, 2 one piece between MFMA groups
    constexpr int MYD = S::NDMA % WAVES == 0 ? S::NDMA / WAVES : 0;
    const int hdma = MYD ? (a.dbg >> 3) & 3 : 0;
    // timing-only skips (x6_dbg bits 2-5 via vdt_set_debug / x6bench; WRONG results): 1 no B DMA
    // past the prologue, 2 no halo reload, 8 no main-loop barriers
    const int hdbg = (a.dbg >> 5) & 15;

    // ---- per-lane A rows: this lane's output row of each fragment i, its halo row for
    // tap (0, 0) and which neighbours exist (bit 0 y-1, 1 y+1, 2 x-1, 3 x+1, 4 row < M)
    int arow[TM], aflg[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
        const int r = wm * S::WTM + i * 16 + (lane & 15), m = m0 + r;
        const int rem = m % HW, y = rem / W, x = rem - y * W;
        arow[i] = r + W + 1;
        aflg[i] = (y > 0 ? 1 : 0) | (y < H - 1 ? 2 : 0) | (x > 0 ? 4 : 0) | (x < W - 1 ? 8 : 0) | (m < a.M ? 16 : 0);
    }

    using AccT = f32x4_t;
    AccT acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = AccT{};
    const int amax_off = std::max(NSB * 2 * PL_B + 2 * PL_H, S::EPR * S::EPLD * 4);
    if (a.ymax)
        for (int f = tid; f < a.B; f += NT) ((unsigned*)(smem + amax_off))[f] = 0u;

    auto compute = [&](int st, int dy, int dx, int dstep) {
        const char* Bs = smem + st * 2 * PL_B;
        const int ch = lane >> 4;
        // S2: taps with d = +1 read the phase pixel itself (its own frame; odd rows / columns
        // past the input were loaded as zeros), d = -1 the previous phase row / column
        const int need = S2 ? (dy < 0 ? 1 : 0) | (dx < 0 ? 4 : 0) | 16
                            : (dy < 0 ? 1 : 0) | (dy > 0 ? 2 : 0) | (dx < 0 ? 4 : 0) | (dx > 0 ? 8 : 0) | 16;
        const int shift = S2 ? (dy < 0 ? -W : 0) + (dx < 0 ? -1 : 0) : dy * W + dx;
        if constexpr (TN < TM) {   // narrow N: B fragments resident, A streamed (VGPRs at 4 waves / SIMD)
            u32x4 bf[TN][3];
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                bf[j][0] = *(const u32x4*)(Bs + swz(wn * S::WTN + j * 16 + (lane & 15), ch));
                bf[j][1] = *(const u32x4*)(Bs + PL_B + swz(wn * S::WTN + j * 16 + (lane & 15), ch));
            }
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                const int hr = (aflg[i] & need) == need ? arow[i] + shift : HR;
                const int o = swzh(hr, ch);
                u32x4 af[3];
                af[0] = *(const u32x4*)(Ah + o);
                af[1] = *(const u32x4*)(Ah + PL_H + o);
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    if constexpr (TR) acc[i][j] = mfma_pair_tr(af, bf[j], acc[i][j]);
                    else acc[i][j] = mfma_terms<2>(af, bf[j], acc[i][j]);
                }
            }
        } else if constexpr (PF) {
            // PF (option x6_halo_pf): the B fragments of column block j + 1 are read before
            // the MFMAs of block j (two buffers: the registers of the compiler's paired reads),
            // pinned by scheduling groups, so an LDS read's latency hides behind 3 TM MFMAs
            u32x4 af[TM][3], bq[2][3];
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                const int hr = (aflg[i] & need) == need ? arow[i] + shift : HR;
                const int o = swzh(hr, ch);
                af[i][0] = *(const u32x4*)(Ah + o);
                af[i][1] = *(const u32x4*)(Ah + PL_H + o);
            }
            bq[0][0] = *(const u32x4*)(Bs + swz(wn * S::WTN + (lane & 15), ch));
            bq[0][1] = *(const u32x4*)(Bs + PL_B + swz(wn * S::WTN + (lane & 15), ch));
            __builtin_amdgcn_sched_group_barrier(0x0100, 2 * TM + 2, 0);
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                if (j + 1 < TN) {
                    bq[(j + 1) & 1][0] = *(const u32x4*)(Bs + swz(wn * S::WTN + (j + 1) * 16 + (lane & 15), ch));
                    bq[(j + 1) & 1][1] = *(const u32x4*)(Bs + PL_B + swz(wn * S::WTN + (j + 1) * 16 + (lane & 15), ch));
                    __builtin_amdgcn_sched_group_barrier(0x0100, 2, 0);
                }
#pragma unroll
                for (int i = 0; i < TM; ++i) {
                    if constexpr (TR) acc[i][j] = mfma_pair_tr(af[i], bq[j & 1], acc[i][j]);
                    else acc[i][j] = mfma_terms<2>(af[i], bq[j & 1], acc[i][j]);
                }
                __builtin_amdgcn_sched_group_barrier(0x0008, 3 * TM, 0);
                if constexpr (MYD > 0 && TN % MYD == 0) {   // x6_halo_dma = 2: a DMA piece per group
                    if (dstep >= 0 && j % (TN / MYD) == 0) dma_piece(dstep, dstep % NSB, j / (TN / MYD));
                }
            }
        } else {
            u32x4 af[TM][3];
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                const int hr = (aflg[i] & need) == need ? arow[i] + shift : HR;
                const int o = swzh(hr, ch);
                af[i][0] = *(const u32x4*)(Ah + o);
                af[i][1] = *(const u32x4*)(Ah + PL_H + o);
            }
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                u32x4 bf[3];
                bf[0] = *(const u32x4*)(Bs + swz(wn * S::WTN + j * 16 + (lane & 15), ch));
                bf[1] = *(const u32x4*)(Bs + PL_B + swz(wn * S::WTN + j * 16 + (lane & 15), ch));
#pragma unroll
                for (int i = 0; i < TM; ++i) {
                    if constexpr (TR) acc[i][j] = mfma_pair_tr(af[i], bf, acc[i][j]);
                    else acc[i][j] = mfma_terms<2>(af[i], bf, acc[i][j]);
                }
                if constexpr (MYD > 0 && TN % MYD == 0) {   // x6_halo_dma = 2: a DMA piece per group
                    if (dstep >= 0 && j % (TN / MYD) == 0) dma_piece(dstep, dstep % NSB, j / (TN / MYD));
                }
            }
        }
    };

    // ---- prologue: chunk 0's halo in LDS (+ the zero row), B of steps 0 and 1 in flight,
    // chunk 1's halo loading into registers
    load_halo(0);
    store_halo();
    if (tid < 8) *(u32x4*)(Ah + (tid >> 2) * PL_H + swzh(HR, tid & 3)) = u32x4{0u, 0u, 0u, 0u};
    dma_b(0, 0);
    const bool one_bar = NSB == 2 && MYD > 0 && !(a.dbg & 4096);
    if (nsteps > 1 && !one_bar) dma_b(1, 1);
    if (nhalo > 1) load_halo(1);
    // Per thread VMEM issue order: ... [halo loads of chunk c+2 at the end of step
    // 9c+8], B(s+2) at the end of step s. At the top of step s, younger than B(s):
    // B(s+1) (if issued) and the halo loads issued at the end of step s-1 or (s = 1)
    // in the prologue after B(1).
    if constexpr (NSB == 3 && S::NDMA % WAVES == 0) {
        // This wave's DMA count per step is a compile-time constant, so each step's vmcnt
        // is one of four immediates chosen by two uniform branches (the runtime wait_vm
        // switch costs a tree of scalar branches per step). (Unrolling the nine taps of a
        // chunk as well measured no better and spills on the 192 / 256-wide tiles.)
        int hcur = 0;                                    // the halo in LDS
        for (int s = 0; s < nsteps; ++s) {
            const int tap = s % 9;
            // halo loads younger than B(s): halo hcur+1's, issued at the end of step s-1 when
            // that step ended a halo, or in the prologue after B(1) (s = 0, 1)
            const bool ended = s >= 1 && (S2 ? s2_last(tap == 0 ? 8 : tap - 1) : tap == 0);
            const bool halo_prev = ended ? hcur + 1 < nhalo : (s <= 1 && nhalo > 1);
            if (halo_prev) {
                if (s + 1 < nsteps) wait_vm_k<MYD + 2 * QI>();
                else wait_vm_k<2 * QI>();
            } else {
                if (s + 1 < nsteps) wait_vm_k<MYD>();
                else wait_vm_k<0>();
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if (!(hdbg & 8)) __builtin_amdgcn_s_barrier();   // B(s) visible; stage (s + 2) % 3 free
            asm volatile("" ::: "memory");
            const bool rehalo = (S2 ? s2_last(tap) : tap == 8) && hcur + 1 < nhalo;
            const bool dnext = !rehalo && s + 2 < nsteps && !(hdbg & 1);
            const int hd = (TN % (MYD ? MYD : 1) == 0 && TN >= TM) ? hdma : (hdma ? 1 : 0);
            if (dnext && hd == 0) dma_b(s + 2, (s + 2) % 3);
            const int wt = S2 ? s2_tap(tap) : tap;
            const int dy = wt / 3 - 1, dx = wt - (wt / 3) * 3 - 1;
            compute(s % 3, dy, dx, dnext && hd == 2 ? s + 2 : -1);
            if (dnext && hd == 1) dma_b(s + 2, (s + 2) % 3);
            if (rehalo) {
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                if (!(hdbg & 8)) __builtin_amdgcn_s_barrier();   // every wave is done with halo hcur
                asm volatile("" ::: "memory");
                if (!(hdbg & 2)) store_halo();
                ++hcur;
                if (hcur + 1 < nhalo && !(hdbg & 2)) load_halo(hcur + 1);
                if (s + 2 < nsteps && !(hdbg & 1)) dma_b(s + 2, (s + 2) % 3);
            }
        }
    } else if constexpr (NSB == 3) {
        // VMEM issue order per step s: [top] B(s+2), except on tap-8 steps, which issue
        // it at the end, after the halo loads of chunk c+2 (the halo stores then wait
        // only on B(s+1), issued a step earlier, not on a DMA just issued). Younger than
        // B(s) at the top of s: B(s+1) and the halo loads issued at the end of s-1 (the
        // prologue's chunk-1 loads follow B(1), so for s = 0 and 1 too).
        for (int s = 0; s < nsteps; ++s) {
            const int c = s / 9, tap = s - 9 * c;
            const bool halo_prev = (s >= 1 && (s - 1) % 9 == 8 && (s - 1) / 9 + 2 < CH) || (s <= 1 && CH > 1);
            const int younger = (s + 1 < nsteps ? my_dma : 0) + (halo_prev ? 2 * QI : 0);
            wait_vm(younger);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();                // B(s) visible; stage (s + 2) % 3 free
            asm volatile("" ::: "memory");
            const bool rehalo = tap == 8 && c + 1 < CH;
            if (!rehalo && s + 2 < nsteps) dma_b(s + 2, (s + 2) % 3);
            const int dy = tap / 3 - 1, dx = tap - (tap / 3) * 3 - 1;
            compute(s % 3, dy, dx, -1);
            if (rehalo) {
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_s_barrier();            // every wave is done with chunk c's halo
                asm volatile("" ::: "memory");
                store_halo();
                if (c + 2 < CH) load_halo(c + 2);
                if (s + 2 < nsteps) dma_b(s + 2, (s + 2) % 3);
            }
        }
    } else if (MYD > 0 && !(a.dbg & 4096)) {
        // two B stages, ONE barrier per step (option x6_halo_1b): B(s+1)'s DMA is issued
        // after step s's barrier (its stage was last read by step s-1, which every wave has
        // finished there); a halo refill (tap 8) takes a second barrier. Younger than B(s)
        // at the top of s: the halo loads issued at the end of step s-1 (or in the prologue,
        // s = 0), behind the refill barrier's memory clobbers.
        int hcur = 0;
        for (int s = 0; s < nsteps; ++s) {
            const int tap = s % 9;
            const bool halo_prev = s == 0 ? nhalo > 1 : (tap == 0 && hcur + 1 < nhalo);
            if (halo_prev) wait_vm_k<2 * QI>();
            else wait_vm_k<0>();
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if (!(hdbg & 8)) __builtin_amdgcn_s_barrier();   // B(s) visible; stage (s + 1) & 1 free
            asm volatile("" ::: "memory");
            // B(s+1) right after the barrier (one step of latency cover: measured 3-4 % faster
            // on the 256-wide tiles than pieces between the MFMA groups, r06t)
            if (s + 1 < nsteps && !(hdbg & 1)) dma_b(s + 1, (s + 1) & 1);
            const int dy = tap / 3 - 1, dx = tap - (tap / 3) * 3 - 1;
            compute(s & 1, dy, dx, -1);
            if (tap == 8 && hcur + 1 < nhalo) {
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                if (!(hdbg & 8)) __builtin_amdgcn_s_barrier();   // every wave is done with halo hcur
                asm volatile("" ::: "memory");
                if (!(hdbg & 2)) store_halo();
                ++hcur;
                if (hcur + 1 < nhalo && !(hdbg & 2)) load_halo(hcur + 1);
            }
        }
    } else {
    for (int s = 0; s < nsteps; ++s) {
        const int c = s / 9, tap = s - 9 * c;
        int younger = s + 1 < nsteps ? my_dma : 0;
        if (s == 0 && CH > 1) younger += 2 * QI;
        if (s == 1 && CH > 1) younger = 2 * QI + (s + 1 < nsteps ? my_dma : 0);
        if (s >= 2 && tap == 0 && c + 1 < CH) younger += 2 * QI;
        wait_vm(younger);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        const int dy = tap / 3 - 1, dx = tap - (tap / 3) * 3 - 1;
        compute(s & 1, dy, dx, -1);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();                    // stage s & 1 (and, at tap 8, the halo) are free
        asm volatile("" ::: "memory");
        if (tap == 8 && c + 1 < CH) {
            store_halo();                                // chunk c+1 (its loads were issued 9 steps ago)
            if (c + 2 < CH) load_halo(c + 2);
        }
        if (s + 2 < nsteps) dma_b(s + 2, s & 1);
    }
    }
    if constexpr (TR) {
        if (a.dbg & 512) x6_epilogue_tr_r5<S>(a, acc, m0, n0, wm, wn, lane, (unsigned*)(smem + amax_off));
        else x6_epilogue_tr<S>(a, acc, m0, n0, wm, wn, lane, (unsigned*)(smem + amax_off));
    } else {
        __syncthreads();
        x6_epilogue<S, 16>(a, acc, m0, n0, wm, wn, tid, lane, smem, amax_off);
    }
}

// ---------------------------------------------------------------------------
// Streaming 1x1 form for the memory-bound bottleneck convs (K = Cin in {64, 128,
// 256}): the split weight slice of NCH output channels sits in LDS for the whole
// (persistent) workgroup, and every wave streams groups of 16 output pixels with
// no workgroup barrier, so loads, MFMAs and stores of the CU's waves interleave.
// D^T[n][p] = sum_k W[n][k] X[p][k]: A = weight rows (LDS, split planes), B = the
// 16 pixels' 8 channels per lane loaded as 2 x 16 B f32 straight from NHWC and
// split in registers; weight rows are permuted so tiles 2i, 2i+1 give a lane 8
// consecutive output channels (two 16-B f32 stores, residual read in the same shape).
//
// TAPS form (round 4, the YOLO net's narrow KxK layers, K <= 288): each lane's 8-channel
// K chunk of every k-step is one (dy, dx, c) of the filter, fixed per lane, so the
// tap table sits in registers; a pixel's chunk is loaded through a buffer descriptor
// (off the frame -> zeros, conv padding) for every k-step. TERMS = 1: integer-valued
// input (x_exact canvases) on one plane against both weight planes. NTT = 1: 16
// output channels, a lane stores 4 consecutive ones.
// RL (round 6, option x6_stream_rl; plain 1x1 form only): the next group's input refills
// each k-step's registers right after that k-step is split (one register set instead of
// two), and the registers saved carry this group's residual, loaded at the top of the
// group beside the MFMAs instead of in the epilogue where its latency stood exposed.
template <int KS, int NTT, int ACT, int RES, int TERMS, bool TAPS = false, bool RL = false>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(TAPS ? 4 : 1)))   // TAPS: two workgroups per CU
void conv1x1_x6_kernel(ConvArgs a, int nchunks, int groups) {
    static_assert(!(RL && (TAPS || NTT == 1)), "RL: the plain 1x1 form with 8-channel lanes");
    constexpr int WT = TERMS == 1 ? 2 : TERMS;             // weight planes
    constexpr int NCH = 16 * NTT, PL = KS * NCH * 64;     // bytes per weight plane
    extern __shared__ __attribute__((aligned(16))) char smem[];
    float* s_scale = (float*)(smem + WT * PL);
    float* s_shift = s_scale + NCH;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int bid = blockIdx.x, xcd = bid & 7, local = bid >> 3;
    const int chunk = local % nchunks;
    const int mblk = (local / nchunks) * 8 + xcd;
    const int nmblk = gridDim.x / nchunks;
    const int n0 = chunk * NCH;
    {   // split weights [n0, n0 + NCH) x K -> LDS [plane][ks][row][64 B]; row 16j + i holds
        // channel 32(j>>1) + 8(i>>2) + 4(j&1) + (i&3)
        const int nk = a.kpad / KT;
        for (int i = tid; i < WT * KS * NCH * 4; i += 512) {
            const int c = i & 3, row = (i >> 2) % NCH, pk = (i >> 2) / NCH, ks = pk % KS, p = pk / KS;
            const int j = row >> 4, ii = row & 15;
            const int chn = NTT == 1 ? row : 32 * (j >> 1) + 8 * (ii >> 2) + 4 * (j & 1) + (ii & 3);
            const u32x4 v = *(const u32x4*)((const char*)a.wx3 + ((((size_t)(n0 + chn) * nk + ks) * WT + p) * 64 + c * 16));
            *(u32x4*)(smem + p * PL + ks * NCH * 64 + swz(row, c)) = v;
        }
        for (int i = tid; i < NCH; i += 512) {
            s_scale[i] = a.scale[n0 + i];
            s_shift[i] = a.shift[n0 + i];
        }
    }
    unsigned* s_amax = (unsigned*)(s_shift + NCH);        // per-frame max |y| (a.ymax)
    if (a.ymax)
        for (int f = tid; f < a.B; f += 512) s_amax[f] = 0u;
    __syncthreads();
    const int p_lane = lane & 15, q = lane >> 4;
    const int ohw = a.yh * a.yw;
    const int wstride = nmblk * 8;
    // TAPS: this lane's (dy, dx, c) per k-step; a chunk past K gets dy far off the frame
    int tdy[TAPS ? KS : 1], tdx[TAPS ? KS : 1], toff[TAPS ? KS : 1];
    if constexpr (TAPS) {
        const int kreal = a.kh * a.kw * a.cin_pad;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            const int k = ks * 32 + q * 8, t = k / a.cin_pad, c = k - t * a.cin_pad;
            const int dy = t / a.kw, dx = t - dy * a.kw;
            tdy[ks] = k < kreal ? dy : (1 << 28);
            tdx[ks] = dx;
            toff[ks] = (dy * a.xw + dx) * a.ldx + c;
        }
    }
    const __amdgpu_buffer_rsrc_t rsrc_x = __builtin_amdgcn_make_buffer_rsrc(
        (void*)a.x, 0, (int)((long)a.B * a.xh * a.xw * a.ldx * 4), 0x00020000);
    auto load = [&](int g, u32x4 (&xf)[KS][2]) {
        const int mu = g * 16 + p_lane;
        const int m = mu < a.M ? mu : a.M - 1;
        const int b = m / ohw, rem = m - b * ohw;
        const int oy = rem / a.yw, ox = rem - oy * a.yw;
        if constexpr (TAPS) {
            const int iy0 = oy * a.stride - a.pad, ix0 = ox * a.stride - a.pad;
            const int pbase = ((b * a.xh + iy0) * a.xw + ix0) * a.ldx + a.xcoff;
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
                const bool ok = ((unsigned)(iy0 + tdy[ks]) < (unsigned)a.xh) & ((unsigned)(ix0 + tdx[ks]) < (unsigned)a.xw);
                const unsigned off = ok ? (unsigned)(pbase + toff[ks]) * 4u : 0x80000000u;
                xf[ks][0] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rsrc_x, (int)off, 0, 0));
                xf[ks][1] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rsrc_x, (int)(off + 16u), 0, 0));
            }
        } else {
            const float* xp = (const float*)a.x + (((size_t)b * a.xh + oy * a.stride) * a.xw + ox * a.stride) * a.ldx +
                              a.xcoff + q * 8;
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
                xf[ks][0] = *(const u32x4*)(xp + ks * 32);
                xf[ks][1] = *(const u32x4*)(xp + ks * 32 + 4);
            }
        }
    };
    (void)rsrc_x;
    u32x4 xf[KS][2];
    int g = mblk * 8 + wid;
    if (g < groups) load(g, xf);
    if constexpr (RL) {
        // pixel m's element offset of its input row (this lane's 8 channels)
        auto xrow = [&](int gg) -> const float* {
            const int mu = gg * 16 + p_lane;
            const int m = mu < a.M ? mu : a.M - 1;
            const int b = m / ohw, rem = m - b * ohw;
            const int oy = rem / a.yw, ox = rem - oy * a.yw;
            return (const float*)a.x + (((size_t)b * a.xh + oy * a.stride) * a.xw + ox * a.stride) * a.ldx + a.xcoff +
                   q * 8;
        };
        // the frame range of the group being split, loaded one group ahead (its load would
        // otherwise sit behind this group's residual loads in the in-order vmcnt)
        // (a buffer load, issued whether or not the range slots exist -- num_records 0 then
        // -- so the compiler's count of younger ops stays exact)
        const __amdgpu_buffer_rsrc_t rsrc_m =
            __builtin_amdgcn_make_buffer_rsrc((void*)a.xmax, 0, a.xmax ? a.B * 4 : 0, 0x00020000);
        auto frame_max = [&](int gg) -> float {
            const int mu = gg * 16 + p_lane;
            const int f = (mu < a.M ? mu : a.M - 1) / ohw;
            const float v = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rsrc_m, f * 4, 0, 0));
            return a.xmax ? v : a.xbound;
        };
        float xm_cur = g < groups ? frame_max(g) : 0.f;
        const __amdgpu_buffer_rsrc_t rsrc_r = __builtin_amdgcn_make_buffer_rsrc(
            (void*)a.res, 0, RES != VD_RES_NONE ? (int)std::min<long>((long)a.M * a.res_ld * 4, 0x7fffffffL) : 0,
            0x00020000);
        for (; g < groups; g += wstride) {
            asm volatile("" ::: "memory");
            const int gn = g + wstride;
            const float* xpn = xrow(gn < groups ? gn : g);
            const float xm_next = frame_max(gn < groups ? gn : g);   // unconditional: straight-line vmcnt
            const int mu = g * 16 + p_lane;
            const int mcl = mu < a.M ? mu : a.M - 1;
            // this group's residual rows, in flight under the MFMAs
            float4 rr[NTT / 2][2];
            if constexpr (RES != VD_RES_NONE) {
                size_t roff;
                if (a.res_up) {
                    const int b = mcl / ohw, rem = mcl - b * ohw;
                    const int oy = rem / a.yw, ox = rem - oy * a.yw;
                    roff = ((size_t)(b * a.rh + (oy >> 1)) * a.rw + (ox >> 1)) * a.res_ld;
                } else {
                    roff = (size_t)mcl * a.res_ld;
                }
                roff += a.res_coff + n0 + q * 8;
                // buffer loads (rows past M read zeros): unconditional, issued here, not sunk
                // into the epilogue where their latency would stand exposed again
                const bool okr = mu < a.M;
#pragma unroll
                for (int i = 0; i < NTT / 2; ++i) {
                    const unsigned o = okr ? (unsigned)((roff + 32 * i) * 4) : 0x80000000u;
                    rr[i][0] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rsrc_r, (int)o, 0, 0));
                    rr[i][1] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rsrc_r, (int)o, 16, 0));
                }
                __builtin_amdgcn_sched_barrier(0);
            }
            f32x4_t acc[NTT];
#pragma unroll
            for (int j = 0; j < NTT; ++j) acc[j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
            const int fb = mcl / ohw;
            const int kexp = TERMS == 2 ? act_scale_exp_of(xm_cur) : 0;
            const float sa = __builtin_ldexpf(1.f, kexp), inv_sa = __builtin_ldexpf(1.f, -kexp);
            xm_cur = xm_next;
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
                float e8[8];
#pragma unroll
                for (int e = 0; e < 8; ++e) e8[e] = __uint_as_float(xf[ks][e >> 2][e & 3]);
                u32x4 xb[3];
                split_pack<TERMS>(e8, sa, xb);
                // refill this k-step's registers with the next group's (the last group re-reads
                // its own rows: no branch, so the compiler counts vmcnt exactly)
                xf[ks][0] = *(const u32x4*)(xpn + ks * 32);
                xf[ks][1] = *(const u32x4*)(xpn + ks * 32 + 4);
#pragma unroll
                for (int j = 0; j < NTT; ++j) {
                    u32x4 wf[3];
#pragma unroll
                    for (int p = 0; p < WT; ++p)
                        wf[p] = *(const u32x4*)(smem + p * PL + ks * NCH * 64 + swz(16 * j + p_lane, q));
                    acc[j] = mfma_terms<TERMS>(wf, xb, acc[j]);
                }
            }
            float vmax = 0.f;
            if (mu < a.M) {
                const size_t yo = (size_t)mu * a.ldy + a.ycoff + n0 + q * 8;
#pragma unroll
                for (int i = 0; i < NTT / 2; ++i) {
                    const int c = 32 * i + q * 8;
                    const float4 s0 = *(const float4*)(s_scale + c), s1 = *(const float4*)(s_scale + c + 4);
                    const float4 h0 = *(const float4*)(s_shift + c), h1 = *(const float4*)(s_shift + c + 4);
                    const f32x4_t& lo = acc[2 * i];
                    const f32x4_t& hi = acc[2 * i + 1];
                    float v[8] = {(lo[0] * inv_sa) * s0.x + h0.x, (lo[1] * inv_sa) * s0.y + h0.y,
                                  (lo[2] * inv_sa) * s0.z + h0.z, (lo[3] * inv_sa) * s0.w + h0.w,
                                  (hi[0] * inv_sa) * s1.x + h1.x, (hi[1] * inv_sa) * s1.y + h1.y,
                                  (hi[2] * inv_sa) * s1.z + h1.z, (hi[3] * inv_sa) * s1.w + h1.w};
                    float rv[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
                    if constexpr (RES != VD_RES_NONE) {
                        rv[0] = rr[i][0].x; rv[1] = rr[i][0].y; rv[2] = rr[i][0].z; rv[3] = rr[i][0].w;
                        rv[4] = rr[i][1].x; rv[5] = rr[i][1].y; rv[6] = rr[i][1].z; rv[7] = rr[i][1].w;
                    }
#pragma unroll
                    for (int e = 0; e < 8; ++e) {
                        float t = v[e];
                        if constexpr (RES == VD_RES_PRE_ACT) t += rv[e];
                        t = act_apply(t, ACT, a.slope);
                        if constexpr (RES == VD_RES_POST_ACT) t += rv[e];
                        v[e] = t;
                        vmax = fmaxf(vmax, fabsf(t));
                    }
                    *(float4*)((float*)a.y + yo + 32 * i) = make_float4(v[0], v[1], v[2], v[3]);
                    *(float4*)((float*)a.y + yo + 32 * i + 4) = make_float4(v[4], v[5], v[6], v[7]);
                }
            }
            if (a.ymax) amax_lds_add(s_amax, mu < a.M ? fb : -1, vmax);
        }
        if (a.ymax) {
            __syncthreads();
            amax_lds_flush(s_amax, a.ymax, a.B);
        }
        return;
    }
    for (; g < groups; g += wstride) {
        asm volatile("" ::: "memory");
        u32x4 xn[KS][2];
        const int gn = g + wstride;
        if (gn < groups) load(gn, xn);
        f32x4_t acc[NTT];
#pragma unroll
        for (int j = 0; j < NTT; ++j) acc[j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
        const int mu = g * 16 + p_lane;
        const int fb = (mu < a.M ? mu : a.M - 1) / ohw;     // this lane's pixel's frame
        const int kexp = TERMS == 2 ? act_scale_exp(a, fb) : 0;
        const float sa = __builtin_ldexpf(1.f, kexp), inv_sa = __builtin_ldexpf(1.f, -kexp);
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            float e8[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) e8[e] = __uint_as_float(xf[ks][e >> 2][e & 3]);
            u32x4 xb[3];
            split_pack<TERMS>(e8, sa, xb);
#pragma unroll
            for (int j = 0; j < NTT; ++j) {
                u32x4 wf[3];
#pragma unroll
                for (int p = 0; p < WT; ++p)
                    wf[p] = *(const u32x4*)(smem + p * PL + ks * NCH * 64 + swz(16 * j + p_lane, q));
                if constexpr (TERMS == 1) {   // w_lo x + w_hi x (x exact on one plane)
                    acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8_t, wf[1]),
                                                                    __builtin_bit_cast(f16x8_t, xb[0]), acc[j], 0, 0, 0);
                    acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8_t, wf[0]),
                                                                    __builtin_bit_cast(f16x8_t, xb[0]), acc[j], 0, 0, 0);
                } else {
                    acc[j] = mfma_terms<TERMS>(wf, xb, acc[j]);
                }
            }
        }
        float vmax = 0.f;
        if (a.dbg & 1) {                                   // timing experiment: no epilogue
            if (acc[0][0] == 1234.5f) ((float*)a.y)[tid] = 1.f;
        } else if (mu < a.M) {
            const int m = mu;
            size_t roff = 0;
            if constexpr (RES != VD_RES_NONE) {
                if (a.res_up) {
                    const int b = m / ohw, rem = m - b * ohw;
                    const int oy = rem / a.yw, ox = rem - oy * a.yw;
                    roff = ((size_t)(b * a.rh + (oy >> 1)) * a.rw + (ox >> 1)) * a.res_ld;
                } else {
                    roff = (size_t)m * a.res_ld;
                }
                roff += a.res_coff + n0 + q * 8;
            }
            if constexpr (NTT == 1) {   // rows = channels: a lane holds channels 4q .. 4q + 3
                if constexpr (RES != VD_RES_NONE) roff -= q * 4;
                const size_t yo1 = (size_t)m * a.ldy + a.ycoff + n0 + q * 4;
                const int c = q * 4;
                float v[4];
                float4 r4 = make_float4(0.f, 0.f, 0.f, 0.f);
                if constexpr (RES != VD_RES_NONE) r4 = *(const float4*)((const float*)a.res + roff);
                const float rv[4] = {r4.x, r4.y, r4.z, r4.w};
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    float t = (acc[0][e] * inv_sa) * s_scale[c + e] + s_shift[c + e];
                    if constexpr (RES == VD_RES_PRE_ACT) t += rv[e];
                    t = act_apply(t, ACT, a.slope);
                    if constexpr (RES == VD_RES_POST_ACT) t += rv[e];
                    v[e] = t;
                    vmax = fmaxf(vmax, fabsf(t));
                }
                *(float4*)((float*)a.y + yo1) = make_float4(v[0], v[1], v[2], v[3]);
            }
            const size_t yo = (size_t)m * a.ldy + a.ycoff + n0 + q * 8;
#pragma unroll
            for (int i = 0; i < NTT / 2; ++i) {
                const int c = 32 * i + q * 8;
                const float4 s0 = *(const float4*)(s_scale + c), s1 = *(const float4*)(s_scale + c + 4);
                const float4 h0 = *(const float4*)(s_shift + c), h1 = *(const float4*)(s_shift + c + 4);
                const f32x4_t& lo = acc[2 * i];
                const f32x4_t& hi = acc[2 * i + 1];
                float v[8] = {(lo[0] * inv_sa) * s0.x + h0.x, (lo[1] * inv_sa) * s0.y + h0.y,
                              (lo[2] * inv_sa) * s0.z + h0.z, (lo[3] * inv_sa) * s0.w + h0.w,
                              (hi[0] * inv_sa) * s1.x + h1.x, (hi[1] * inv_sa) * s1.y + h1.y,
                              (hi[2] * inv_sa) * s1.z + h1.z, (hi[3] * inv_sa) * s1.w + h1.w};
                float rv[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
                if constexpr (RES != VD_RES_NONE) {
                    const float4 r0 = *(const float4*)((const float*)a.res + roff + 32 * i);
                    const float4 r1 = *(const float4*)((const float*)a.res + roff + 32 * i + 4);
                    rv[0] = r0.x; rv[1] = r0.y; rv[2] = r0.z; rv[3] = r0.w;
                    rv[4] = r1.x; rv[5] = r1.y; rv[6] = r1.z; rv[7] = r1.w;
                }
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    float t = v[e];
                    if constexpr (RES == VD_RES_PRE_ACT) t += rv[e];
                    t = act_apply(t, ACT, a.slope);
                    if constexpr (RES == VD_RES_POST_ACT) t += rv[e];
                    v[e] = t;
                    vmax = fmaxf(vmax, fabsf(t));
                }
                *(float4*)((float*)a.y + yo + 32 * i) = make_float4(v[0], v[1], v[2], v[3]);
                *(float4*)((float*)a.y + yo + 32 * i + 4) = make_float4(v[4], v[5], v[6], v[7]);
            }
        }
        if (a.ymax) amax_lds_add(s_amax, mu < a.M ? fb : -1, vmax);
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) { xf[ks][0] = xn[ks][0]; xf[ks][1] = xn[ks][1]; }
    }
    if (a.ymax) {
        __syncthreads();
        amax_lds_flush(s_amax, a.ymax, a.B);
    }
}

// Dual streaming form (fp16 pairs): a bottleneck's conv3 (+bn3) and its downsample
// (+bn, strided 1x1 over the block input) for the same output pixels in one pass,
// y = relu((bn3(conv3(t2))) + bn_d(ds(x))): the downsample output never goes
// through HBM. The two products keep their own per-frame operand scales (t2's and
// x's producers' max), and the downsample term is rounded to f32 before the add as
// the unfused plan stores it, so the result is bit-identical to conv_ds followed by
// conv3 with a pre-activation residual. Layer1.0 (K 64 + 64).
template <int KS, int KS2, int NTT>
__global__ __launch_bounds__(512) void conv1x1_x6_dual_kernel(ConvArgs a, int nchunks, int groups) {
    constexpr int NCH = 16 * NTT, PL = KS * NCH * 64, PL2 = KS2 * NCH * 64;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* w2s = smem + 2 * PL;
    float* s_scale = (float*)(w2s + 2 * PL2);
    float* s_shift = s_scale + NCH;
    float* s_scale2 = s_shift + NCH;
    float* s_shift2 = s_scale2 + NCH;
    unsigned* s_amax = (unsigned*)(s_shift2 + NCH);
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int bid = blockIdx.x, xcd = bid & 7, local = bid >> 3;
    const int chunk = local % nchunks;
    const int mblk = (local / nchunks) * 8 + xcd;
    const int nmblk = gridDim.x / nchunks;
    const int n0 = chunk * NCH;
    auto stage_w = [&](const void* wsrc, int kpad, int ks_n, char* dst, int pl) {
        const int nk = kpad / KT;
        for (int i = tid; i < 2 * ks_n * NCH * 4; i += 512) {
            const int c = i & 3, row = (i >> 2) % NCH, pk = (i >> 2) / NCH, ks = pk % ks_n, p = pk / ks_n;
            const int j = row >> 4, ii = row & 15;
            const int chn = 32 * (j >> 1) + 8 * (ii >> 2) + 4 * (j & 1) + (ii & 3);
            const u32x4 v = *(const u32x4*)((const char*)wsrc + ((((size_t)(n0 + chn) * nk + ks) * 2 + p) * 64 + c * 16));
            *(u32x4*)(dst + p * pl + ks * NCH * 64 + swz(row, c)) = v;
        }
    };
    stage_w(a.wx3, a.kpad, KS, smem, PL);
    stage_w(a.wx3_2, a.kpad2, KS2, w2s, PL2);
    for (int i = tid; i < NCH; i += 512) {
        s_scale[i] = a.scale[n0 + i];
        s_shift[i] = a.shift[n0 + i];
        s_scale2[i] = a.scale2[n0 + i];
        s_shift2[i] = a.shift2[n0 + i];
    }
    if (a.ymax)
        for (int f = tid; f < a.B; f += 512) s_amax[f] = 0u;
    __syncthreads();
    const int p_lane = lane & 15, q = lane >> 4;
    const int ohw = a.yh * a.yw;
    const int wstride = nmblk * 8;
    auto load = [&](int g, u32x4 (&xf)[KS][2], u32x4 (&xf2)[KS2][2]) {
        const int mu = g * 16 + p_lane;
        const int m = mu < a.M ? mu : a.M - 1;
        const int b = m / ohw, rem = m - b * ohw;
        const int oy = rem / a.yw, ox = rem - oy * a.yw;
        const float* xp = (const float*)a.x + (((size_t)b * a.xh + oy * a.stride) * a.xw + ox * a.stride) * a.ldx +
                          a.xcoff + q * 8;
        const float* xp2 = (const float*)a.x2 +
                           (((size_t)b * a.xh2 + oy * a.stride2) * a.xw2 + ox * a.stride2) * a.ldx2 + a.xcoff2 + q * 8;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            xf[ks][0] = *(const u32x4*)(xp + ks * 32);
            xf[ks][1] = *(const u32x4*)(xp + ks * 32 + 4);
        }
#pragma unroll
        for (int ks = 0; ks < KS2; ++ks) {
            xf2[ks][0] = *(const u32x4*)(xp2 + ks * 32);
            xf2[ks][1] = *(const u32x4*)(xp2 + ks * 32 + 4);
        }
    };
    auto gemm = [&](f32x4_t (&acc)[NTT], const auto& xf, const char* wl, int pl, float sa) {
        constexpr int ks_n = sizeof(xf) / sizeof(xf[0]);
#pragma unroll
        for (int ks = 0; ks < ks_n; ++ks) {
            float e8[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) e8[e] = __uint_as_float(xf[ks][e >> 2][e & 3]);
            u32x4 xb[3];
            split_pack<2>(e8, sa, xb);
#pragma unroll
            for (int j = 0; j < NTT; ++j) {
                u32x4 wf[3];
#pragma unroll
                for (int p = 0; p < 2; ++p) wf[p] = *(const u32x4*)(wl + p * pl + ks * NCH * 64 + swz(16 * j + p_lane, q));
                acc[j] = mfma_terms<2>(wf, xb, acc[j]);
            }
        }
    };
    ConvArgs a2 = a;                                       // the downsample input's range slots
    a2.xmax = a.x2max;
    a2.xbound = a.x2bound;
    u32x4 xf[KS][2], xf2[KS2][2];
    int g = mblk * 8 + wid;
    if (g < groups) load(g, xf, xf2);
    for (; g < groups; g += wstride) {
        asm volatile("" ::: "memory");
        u32x4 xn[KS][2], xn2[KS2][2];
        const int gn = g + wstride;
        if (gn < groups) load(gn, xn, xn2);
        const int mu = g * 16 + p_lane;
        const int fb = (mu < a.M ? mu : a.M - 1) / ohw;
        const int k1 = act_scale_exp(a, fb), k2 = act_scale_exp(a2, fb);
        f32x4_t acc[NTT], acc2[NTT];
#pragma unroll
        for (int j = 0; j < NTT; ++j) acc[j] = acc2[j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
        gemm(acc, xf, smem, PL, __builtin_ldexpf(1.f, k1));
        gemm(acc2, xf2, w2s, PL2, __builtin_ldexpf(1.f, k2));
        const float inv1 = __builtin_ldexpf(1.f, -k1), inv2 = __builtin_ldexpf(1.f, -k2);
        float vmax = 0.f;
        if (mu < a.M) {
            const size_t yo = (size_t)mu * a.ldy + a.ycoff + n0 + q * 8;
#pragma unroll
            for (int i = 0; i < NTT / 2; ++i) {
                const int c = 32 * i + q * 8;
                float v[8];
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    const float a1 = (e < 4 ? acc[2 * i][e] : acc[2 * i + 1][e - 4]);
                    const float a2v = (e < 4 ? acc2[2 * i][e] : acc2[2 * i + 1][e - 4]);
                    const float r = (a2v * inv2) * s_scale2[c + e] + s_shift2[c + e];   // the stored ds value
                    float t = (a1 * inv1) * s_scale[c + e] + s_shift[c + e];
                    t += r;
                    t = t > 0.f ? t : 0.f;
                    v[e] = t;
                    vmax = fmaxf(vmax, t);
                }
                *(float4*)((float*)a.y + yo + 32 * i) = make_float4(v[0], v[1], v[2], v[3]);
                *(float4*)((float*)a.y + yo + 32 * i + 4) = make_float4(v[4], v[5], v[6], v[7]);
            }
        }
        if (a.ymax) amax_lds_add(s_amax, mu < a.M ? fb : -1, vmax);
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) { xf[ks][0] = xn[ks][0]; xf[ks][1] = xn[ks][1]; }
#pragma unroll
        for (int ks = 0; ks < KS2; ++ks) { xf2[ks][0] = xn2[ks][0]; xf2[ks][1] = xn2[ks][1]; }
    }
    if (a.ymax) {
        __syncthreads();
        amax_lds_flush(s_amax, a.ymax, a.B);
    }
}

template <int KS, int KS2, int NTT>
hipError_t launch_dual_x6(const ConvArgs& a0, hipStream_t s) {
    constexpr int NCH = 16 * NTT;
    constexpr int lds = 2 * (KS + KS2) * NCH * 64 + 4 * NCH * 4;
    static const int resident = [] {
        (void)hipFuncSetAttribute((const void*)conv1x1_x6_dual_kernel<KS, KS2, NTT>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, lds + 4 * kAmaxFrames);
        int dev = 0, cus = 256, per_cu = 1;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, conv1x1_x6_dual_kernel<KS, KS2, NTT>, 512, lds);
        return std::max(1, cus * std::max(1, per_cu));
    }();
    ConvArgs a = a0;
    a.scale = a.scale_x;                                   // per-channel rescaled BN scales of the pairs
    a.scale2 = a.scale2_x;
    const int nchunks = a.cout / NCH;
    const int groups = (a.M + 15) / 16;
    int k = std::max(1, resident / (8 * nchunks));
    k = std::min(k, std::max(1, (groups + 63) / 64));
    hipLaunchKernelGGL((conv1x1_x6_dual_kernel<KS, KS2, NTT>), dim3(8 * nchunks * k), dim3(512),
                       lds + (a.ymax ? 4 * a.B : 0), s, a, nchunks, groups);
    return hipGetLastError();
}

template <int KS, int NTT, int ACT, int RES, int TERMS, bool TAPS = false, bool RL = false>
hipError_t launch_stream_x6(const ConvArgs& a, hipStream_t s) {
    // option x6_stream_rl (default 1): the RL form for the layers with a residual (layer3
    // conv3 330 -> 299 us, layer2 conv3 416 -> 404 in x6bench); without one it measured
    // slower (layer2.0 conv1 577 -> 603), so those keep the two-set form
    if constexpr (!TAPS && !RL && NTT >= 2 && TERMS == 2) {
        // x6_stream_rl 2: also the layers without a residual
        if (a.tune && (RES != VD_RES_NONE ? a.tune->x6_stream_rl : a.tune->x6_stream_rl >= 2))
            return launch_stream_x6<KS, NTT, ACT, RES, TERMS, false, true>(a, s);
    }
    constexpr int NCH = 16 * NTT;
    constexpr int lds = (TERMS == 1 ? 2 : TERMS) * KS * NCH * 64 + 2 * NCH * 4;
    static const int resident = [] {
        (void)hipFuncSetAttribute((const void*)conv1x1_x6_kernel<KS, NTT, ACT, RES, TERMS, TAPS, RL>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, lds + 4 * kAmaxFrames);
        int dev = 0, cus = 256, per_cu = 1;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, conv1x1_x6_kernel<KS, NTT, ACT, RES, TERMS, TAPS, RL>,
                                                           512, lds);
        return std::max(1, cus * std::max(1, per_cu));
    }();
    const int nchunks = a.cout / NCH;
    const int groups = (a.M + 15) / 16;
    int k = std::max(1, resident / (8 * nchunks));
    k = std::min(k, std::max(1, (groups + 63) / 64));
    hipLaunchKernelGGL((conv1x1_x6_kernel<KS, NTT, ACT, RES, TERMS, TAPS, RL>), dim3(8 * nchunks * k), dim3(512),
                       lds + (a.ymax ? 4 * a.B : 0), s, a, nchunks, groups);
    return hipGetLastError();
}

// TAPS streaming form (fp16 pairs): the narrow KxK layers of the YOLO net -- Cin a
// multiple of 8, K (padded) <= 160, Cout 16 / 32 as one channel slice, SiLU (the
// C2f bottleneck's shortcut as a post-activation residual) -- and the space-to-depth
// model.0 on its integer canvas (x_exact: one A plane). Returns false when not taken.
static bool launch_taps_x6(const ConvArgs& a, hipStream_t s, hipError_t* err) {
    // plain 1x1 convs go to the streaming form unless their K is padded (model.2's cv2 over
    // the 48-channel C2f concat: K 48 in a 64-wide k range)
    if (!a.tune || !a.tune->x6_taps ||
        (a.kh == 1 && a.kw == 1 && a.pad == 0 && a.stride == 1 && a.kpad == a.cin_pad))
        return false;
    if (a.act != VD_ACT_SILU || (a.res_mode != VD_RES_NONE && a.res_mode != VD_RES_POST_ACT)) return false;
    if ((a.cin_pad & 7) || ((a.ldx | a.xcoff) & 3) || ((a.ldy | a.ycoff) & 7)) return false;
    if (a.res_mode != VD_RES_NONE && (a.res_up || ((a.res_ld | a.res_coff) & 7))) return false;
    if (a.kpad > 160 || a.kpad % 32) return false;
    const int ks = a.kpad / 32, co = a.cout;
    const bool post = a.res_mode == VD_RES_POST_ACT;
#define VD_TAPS(KS, NTT, T)                                                                                        \
    do {                                                                                                           \
        *err = post ? launch_stream_x6<KS, NTT, VD_ACT_SILU, VD_RES_POST_ACT, T, true>(a, s)                       \
                    : launch_stream_x6<KS, NTT, VD_ACT_SILU, VD_RES_NONE, T, true>(a, s);                          \
        return true;                                                                                               \
    } while (0)
    if (a.x_exact) {
        if (ks == 2 && co == 16 && !post) {
            *err = launch_stream_x6<2, 1, VD_ACT_SILU, VD_RES_NONE, 1, true>(a, s);
            return true;
        }
        return false;
    }
    // K <= 160 only: at K = 288 (model.3, the 32-channel bottlenecks at 80x48) the
    // two register sets of x need ~210 VGPRs, one workgroup per CU, and the form
    // measured 5-40 % slower than the GEMM / halo tiles
    if (ks == 2 && co == 32) VD_TAPS(2, 2, 2);
    if (ks == 5 && co == 16) VD_TAPS(5, 1, 2);
    if (ks == 5 && co == 32) VD_TAPS(5, 2, 2);
#undef VD_TAPS
    return false;
}

template <int KS, int NTT, int TERMS>
hipError_t stream_mode_x6(const ConvArgs& a, hipStream_t s) {
    if (a.act == VD_ACT_RELU) {
        if (a.res_mode == VD_RES_PRE_ACT) return launch_stream_x6<KS, NTT, VD_ACT_RELU, VD_RES_PRE_ACT, TERMS>(a, s);
        if (a.res_mode == VD_RES_NONE) return launch_stream_x6<KS, NTT, VD_ACT_RELU, VD_RES_NONE, TERMS>(a, s);
    }
    if (a.act == VD_ACT_NONE && a.res_mode == VD_RES_NONE)
        return launch_stream_x6<KS, NTT, VD_ACT_NONE, VD_RES_NONE, TERMS>(a, s);
    return hipErrorInvalidValue;   // excluded by stream_x6_nch
}

__global__ void amax_merge_kernel(unsigned* dst, const unsigned* src, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) dst[i] = max(dst[i], src[i]);
}

}  // namespace

// max-pool / upsample outputs of the fp16-pair plan: the output's per-frame range is
// within the input's (plate_net.cpp SPPF / Upsample, the f32 face stem's pool)
hipError_t vd_launch_amax_merge(unsigned* dst, const unsigned* src, int n, hipStream_t s) {
    hipLaunchKernelGGL(amax_merge_kernel, dim3((n + 63) / 64), dim3(64), 0, s, dst, src, n);
    return hipGetLastError();
}

// Eligible: f32 activations with Cin padded to 4, K padded to 32, split weights present.
bool vd_conv_x6_ok(const ConvArgs& a) {
    const double xbytes = (double)a.B * a.xh * a.xw * a.ldx * 4;   // 32-bit buffer offsets
    return a.wx3 != nullptr && (a.kpad % KT) == 0 && (a.cin_pad % 4) == 0 && ((a.ldx | a.xcoff) & 3) == 0 &&
           xbytes < 2147483647.0;
}

// rows [mbase, M) of the conv (mbase a multiple of the caller's tile rows)
template <int BM, int BN, int NT, int NST, int TERMS, int MF = 16, int NA = 2, bool TR = false, bool PF = false>
static hipError_t launch_x6(const ConvArgs& a0, hipStream_t s, int mbase = 0, int mtiles = -1) {
    if constexpr (NA == 2 && BM == 256 && BN <= 128 && NST == 2 && TERMS == 2 && MF == 16 && !TR && !PF) {
        // option x6_adepth: four A register sets (three K tiles of A loads in flight) on
        // the 256 x {128, 64, 32} tiles, whose accumulators leave the registers for them
        if (a0.tune && a0.tune->x6_adepth >= 4) return launch_x6<BM, BN, NT, NST, TERMS, MF, 4>(a0, s, mbase, mtiles);
    }
    if constexpr (!PF && MF == 16 && NST == 2 && X6Shape<BM, BN, NT, NST, TERMS, MF>::TN > X6Shape<BM, BN, NT, NST, TERMS, MF>::TM) {
        // option x6_gemm_pf: the wide-wave tiles with pipelined B-fragment reads
        if (a0.tune && a0.tune->x6_gemm_pf) return launch_x6<BM, BN, NT, NST, TERMS, MF, NA, TR, true>(a0, s, mbase, mtiles);
    }
    using S = X6Shape<BM, BN, NT, NST, TERMS, MF>;
    static const bool attr = [] {
        (void)hipFuncSetAttribute((const void*)conv_x6_kernel<BM, BN, NT, NST, TERMS, MF, NA, TR, PF>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, S::LDS + 4 * kAmaxFrames);
        return true;
    }();
    (void)attr;
    ConvArgs a = a0;
    a.w = a.wx3;                                   // the kernel reads the split planes
    a.ntiles_n = (a.cout + BN - 1) / BN;
    a.mbase = mbase;
    const int mt = mtiles >= 0 ? mtiles : (a.M - mbase + BM - 1) / BM;
    const int lds = S::LDS + (a.ymax ? 4 * a.B : 0);
    hipLaunchKernelGGL((conv_x6_kernel<BM, BN, NT, NST, TERMS, MF, NA, TR, PF>), dim3(mt * a.ntiles_n), dim3(NT), lds, s, a);
    return hipGetLastError();
}

static int device_cus() {
    static const int cus = [] {
        int dev = 0, n = 256;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
        return std::max(1, n);
    }();
    return cus;
}

// The 256 x BN two-stage tile runs one workgroup per CU, so a grid of R full rounds
// plus a partial one leaves most CUs idle during the last round (400 tiles of layer3:
// 1.56 rounds on 256 CUs take 2). Tail split: the whole rounds as usual, then the
// remaining rows in one more launch of a narrower tile (BN / 2 or BN / 4 columns),
// 2-4x as many workgroups, each a fraction of the time. Splitting N (never K) leaves
// every output's sum in the same K order on the same MFMA form, so the result is
// bit-identical to the unsplit launch.
template <int BN, int TERMS, int MF = 16>
static hipError_t launch_x6_big(const ConvArgs& a, hipStream_t s) {
    const int tail = a.tune ? a.tune->x6_tail : 0;
    const int nt = (a.cout + BN - 1) / BN, mt = (a.M + 255) / 256;
    const int slots = a.tune && a.tune->x6_slots > 0 ? a.tune->x6_slots : device_cus();
    const long total = (long)mt * nt;
    if (TERMS != 2 || MF != 16 || !tail || total <= slots || total % slots == 0 || slots % nt) {
        return launch_x6<256, BN, 512, 2, TERMS, MF>(a, s);
    }
    const int mt_main = (int)(total / slots) * (slots / nt);
    if (mt_main <= 0 || mt_main >= mt) return launch_x6<256, BN, 512, 2, TERMS, MF>(a, s);
    hipError_t e = launch_x6<256, BN, 512, 2, TERMS, MF>(a, s, 0, mt_main);
    if (e != hipSuccess) return e;
    const int mb = mt_main * 256;
    constexpr int BN1 = BN == 192 ? 64 : BN / 2, BN2 = BN == 192 ? 64 : BN / 4;
    if (tail == 1 || BN2 < 32) return launch_x6<256, BN1, 512, 2, TERMS, MF>(a, s, mb);
    return launch_x6<256, BN2, 512, 2, TERMS, MF>(a, s, mb);
}

template <int BN, int NSB>
static int x6_halo_lds(const ConvArgs& a) {
    using S = X6Shape<256, BN, 512, 2, 2>;
    const int HP = a.stride == 2 ? 256 + a.yw + 2 : 256 + 2 * a.yw + 3;
    return std::max(NSB * 2 * S::PL_B + 2 * HP * 64, S::EPR * S::EPLD * 4) + (a.ymax ? 4 * a.B : 0);
}

template <int BN, int NSB, bool TR, bool S2, bool PF>
static hipError_t launch_x6_halo_pf(const ConvArgs& a0, hipStream_t s) {
    ConvArgs a = a0;
    a.w = a.wx3;
    a.ntiles_n = (a.cout + BN - 1) / BN;
    a.mbase = 0;
    static const bool attr = [] {
        (void)hipFuncSetAttribute((const void*)conv_x6_halo_kernel<BN, NSB, TR, S2, PF>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        return true;
    }();
    (void)attr;
    const int lds = x6_halo_lds<BN, NSB>(a);
    if (lds > 160 * 1024) return hipErrorInvalidValue;
    const int mt = (a.M + 255) / 256;
    hipLaunchKernelGGL((conv_x6_halo_kernel<BN, NSB, TR, S2, PF>), dim3(mt * a.ntiles_n), dim3(512), lds, s, a);
    return hipGetLastError();
}

// option x6_halo_pf: the pipelined B-fragment reads on the 128-256-wide tiles
template <int BN, int NSB, bool TR = false, bool S2 = false>
static hipError_t launch_x6_halo_t(const ConvArgs& a, hipStream_t s) {
    if constexpr (BN >= 128) {
        if (a.tune && a.tune->x6_halo_pf) return launch_x6_halo_pf<BN, NSB, TR, S2, true>(a, s);
    }
    return launch_x6_halo_pf<BN, NSB, TR, S2, false>(a, s);
}

// TR form where the output (and residual) rows take 8-channel 16-B vectors (option
// x6_halo_tr: 1 the 128 / 192 / 256-wide tiles, 2 the narrow ones too)
template <int BN, int NSB>
static hipError_t launch_x6_halo_n(const ConvArgs& a, hipStream_t s) {
    const bool tr = a.tune && a.tune->x6_halo_tr >= (BN >= 128 ? 1 : 2) && !((a.ldy | a.ycoff) & 7) && tr_bytes_ok(a) &&
                    (a.res_mode == VD_RES_NONE || !((a.res_ld | a.res_coff) & 7));
    if constexpr (NSB == 3 && BN >= 64) {   // stride 2: the phase halos (x6_halo_ok)
        if (a.stride == 2) return tr ? launch_x6_halo_t<BN, 3, true, true>(a, s) : launch_x6_halo_t<BN, 3, false, true>(a, s);
    }
    if (a.stride != 1) return hipErrorInvalidValue;
    if (tr) return launch_x6_halo_t<BN, NSB, true>(a, s);
    return launch_x6_halo_t<BN, NSB, false>(a, s);
}

// option x6_halo: 1 two B stages, 2 three where they fit LDS beside the halo
template <int BN>
static hipError_t launch_x6_halo(const ConvArgs& a, hipStream_t s) {
    if ((a.tune->x6_halo >= 2 || a.stride == 2) && x6_halo_lds<BN, 3>(a) <= 160 * 1024) return launch_x6_halo_n<BN, 3>(a, s);
    return launch_x6_halo_n<BN, 2>(a, s);
}

// 3x3 / stride 1 / pad 1, same-size in and out, K = 9 x Cin in whole 32-channel chunks,
// halo of at most 512 rows (W <= 126) that fits LDS beside the B stages; stride 2 (option
// x6_halo_s2): the phase halos of at most 512 rows (Wo <= 254), N tiles of >= 64 (Cout > 32,
// whole DMA rounds), three B stages, dense
static bool x6_halo_ok(const ConvArgs& a) {
    if (!a.tune || !a.tune->x6_halo || a.kh != 3 || a.kw != 3 || a.pad != 1) return false;
    if (a.cin_pad % 32 || a.kpad != 9 * a.cin_pad || (a.ymax && a.B > kAmaxFrames)) return false;
    if (a.stride == 2) {
        if (!a.tune->x6_halo_s2 || a.cout <= 32 || a.grp_co) return false;
        if (a.yh != (a.xh - 1) / 2 + 1 || a.yw != (a.xw - 1) / 2 + 1 || 256 + a.yw + 2 > 512) return false;
        return (3 * 2 * 256 * 64 + 2 * (256 + a.yw + 2) * 64 + (a.ymax ? 4 * a.B : 0)) <= 160 * 1024;
    }
    if (a.stride != 1 || a.xh != a.yh || a.xw != a.yw) return false;
    if (256 + 2 * a.yw + 2 > 512) return false;
    return true;
}

// N tile follows Cout (weights are packed with Npad a multiple of 128, so every
// tile's rows exist): 32 for the heads, 64 for the 64-channel convs, else 128.
// The small single-stage tile takes the narrow (N <= 64) layers with K <= 256 or
// a grid of fewer than 512 big tiles (measured: stem 2.16 -> 1.87 ms, layer1 conv1
// 640 -> 580 us, SSH level 1/2 and heads 15-25 % faster); at N = 128 it measured
// 30-45 % slower than the big tile (one wave per SIMD at 198 VGPRs) and is not used.
// Streaming 1x1 (conv1x1_x6_kernel): 1x1 taps without padding, K = Cin in {64, 128,
// 256} (one channel slice of 128, or 64 at K = 256, fits 96 KB of LDS in three split
// planes), ReLU with / without the pre-activation residual, or no activation.
static int stream_x6_nch(const ConvArgs& a, int terms) {
    if (!a.tune || !a.tune->x6_stream || a.kh != 1 || a.kw != 1 || a.pad != 0 || a.kpad != a.cin_pad) return 0;
    if (a.cin_pad != 64 && a.cin_pad != 128 && a.cin_pad != 256) return 0;
    const bool mode = (a.act == VD_ACT_RELU && (a.res_mode == VD_RES_NONE || a.res_mode == VD_RES_PRE_ACT)) ||
                      (a.act == VD_ACT_NONE && a.res_mode == VD_RES_NONE);
    if (!mode || ((a.ldx | a.xcoff | a.ldy | a.ycoff) & 7)) return 0;
    if (a.res_mode != VD_RES_NONE && ((a.res_ld | a.res_coff) & 7)) return 0;
    const int nch = (a.cin_pad == 256 && terms == 3) ? 64 : 128;
    if (a.cout % nch == 0) return nch;
    return a.cout % 64 == 0 && a.cin_pad <= 128 ? 64 : 0;
}

// TR tiles (option x6_gemm1x1, default): the 1x1 convs the streaming form does not take
// (K >= 512, strided downsamples) on conv_x6_kernel with D^T accumulators and the
// register epilogue (x6_epilogue_tr). Same tiles and products as the untransposed form,
// bit-identical results (tests/test_gpu_kernels.py); the epilogue skips the LDS round
// trip and its two barriers per pass (tools/x6bench, B = 64: layer4 conv3 334 -> 304 us,
// layer3.0 downsample 528 -> 472, layer3 conv1 263 -> 243, FPN output1 553 -> 512).
// Measured and not kept: the pixel operand loaded straight into registers by the two
// waves of its row band (no LDS image, one barrier per K tile with three weight
// stages): its main loop ran 5-10 % slower than the LDS-staged one (layer3 conv1
// 215 -> 235 us without epilogue). Needs 8-channel 16-B output / residual vectors.
static bool x6_tr_ok(const ConvArgs& a) {
    if (a.kh != 1 || a.kw != 1 || a.pad != 0 || a.cout % 128 || !tr_bytes_ok(a)) return false;
    if ((a.ldy | a.ycoff) & 7) return false;
    return a.res_mode == VD_RES_NONE || !((a.res_ld | a.res_coff) & 7);
}

static hipError_t launch_tr(const ConvArgs& a, hipStream_t s) {
    const long t256 = (long)((a.M + 255) / 256) * (a.cout / 256);
    // (Measured and not kept, round 6: Cout >= 512 1x1 layers with K <= 512-2048 on the
    // 128 x 128 tile at two workgroups per CU -- level to 8 % slower, tools/runs/r06y.sh)
    if (a.cout % 256 == 0 && t256 >= 192) return launch_x6<256, 256, 512, 2, 2, 16, 2, true>(a, s);
    if (a.cout == 128 && a.tune->x6_mid && a.kpad <= a.tune->x6_mid) return launch_x6<128, 128, 256, 2, 2, 16, 2, true>(a, s);
    return launch_x6<256, 128, 512, 2, 2, 16, 2, true>(a, s);
}

template <int TERMS>
static hipError_t launch_terms(const ConvArgs& a0, hipStream_t s) {
    ConvArgs a = a0;
    if (TERMS == 2) a.scale = a.scale_x;              // the fp16 pair's per-channel rescaled BN scale
    if constexpr (TERMS == 2) {
        hipError_t err = hipSuccess;
        if (launch_taps_x6(a, s, &err)) return err;
    }
    if constexpr (TERMS == 2) {   // YOLO's SiLU 1x1 convs (C2f cv1 / cv2, SPPF cv1) on the streaming form
        if (a.tune && a.tune->x6_stream_silu && a.act == VD_ACT_SILU && a.res_mode == VD_RES_NONE && a.kh == 1 &&
            a.kw == 1 && a.pad == 0 && a.kpad == a.cin_pad && !((a.ldx | a.xcoff | a.ldy | a.ycoff) & 7)) {
            const int k = a.cin_pad, co = a.cout;
            const int nch = co % 128 == 0 ? 128 : (co % 64 == 0 ? 64 : (co % 32 == 0 ? 32 : 0));
            if (nch) {
#define VD_SILU(KS, NTT) return launch_stream_x6<KS, NTT, VD_ACT_SILU, VD_RES_NONE, 2>(a, s)
                if (k == 32 && nch == 32) VD_SILU(1, 2);
                if (k == 32 && nch == 64) VD_SILU(1, 4);
                if (k == 64 && nch == 64) VD_SILU(2, 4);
                if (k == 64 && nch == 128) VD_SILU(2, 8);
                if (k == 96 && nch == 64) VD_SILU(3, 4);
                if (k == 128 && nch == 64) VD_SILU(4, 4);
                if (k == 128 && nch == 128) VD_SILU(4, 8);
                if (k == 192 && nch == 64) VD_SILU(6, 4);
                if (k == 192 && nch == 128) VD_SILU(6, 8);
                if (k == 256 && nch == 128) VD_SILU(8, 8);
#undef VD_SILU
            }
        }
    }
    if constexpr (TERMS == 2) {
        // option x6_gemm1x1 = 2 (experiments): the K <= 256 layers of the streaming form on the
        // TR tiles as well (measured 20-35 % slower than the streaming form)
        if (a.tune && a.tune->x6_gemm1x1 == 2 && x6_tr_ok(a)) return launch_tr(a, s);
    }
    if (const int nch = stream_x6_nch(a, TERMS)) {
        if constexpr (TERMS == 2) {   // 256-channel slices: each pixel read by half as many workgroups
            if (a.tune && a.tune->x6_stream256 && a.cout % 256 == 0) {
                if (a.cin_pad == 64) return stream_mode_x6<2, 16, TERMS>(a, s);
                if (a.cin_pad == 128 && a.tune->x6_stream256 > 1) return stream_mode_x6<4, 16, TERMS>(a, s);   // 128 KB LDS
            }
        }
        if (a.cin_pad == 64) return nch == 128 ? stream_mode_x6<2, 8, TERMS>(a, s) : stream_mode_x6<2, 4, TERMS>(a, s);
        if (a.cin_pad == 128) return nch == 128 ? stream_mode_x6<4, 8, TERMS>(a, s) : stream_mode_x6<4, 4, TERMS>(a, s);
        if constexpr (TERMS == 2) return stream_mode_x6<8, 8, TERMS>(a, s);
        return stream_mode_x6<8, 4, TERMS>(a, s);
    }
    if constexpr (TERMS == 2) {
        if (a.tune && a.tune->x6_gemm1x1 && x6_tr_ok(a)) return launch_tr(a, s);
    }
    const int bn = a.cout <= 32 ? 32 : (a.cout <= 64 ? 64 : 128);
    const long big_tiles = (long)((a.M + 255) / 256) * ((a.cout + bn - 1) / bn);
    const int small_k = a.tune ? a.tune->x6_small_k : 256, small_tiles = a.tune ? a.tune->x6_small_tiles : 512;
    const int small_k2 = a.tune ? a.tune->x6_small_k2 : (1 << 20);
    const bool force_small = small_k >= (1 << 30);       // test hook: every layer on the small tile
    // fp16 pairs: the 4-wave one-stage tile wins for every N <= 64 layer measured
    // (layer1 conv2 831 -> 603 us, SSH level-0 conv7X7 229 -> 163 us)
    const bool small = force_small || (bn <= 64 && (a.kpad <= (TERMS == 2 ? small_k2 : small_k) ||
                                                    big_tiles < small_tiles));
    if constexpr (TERMS == 2) {   // narrow 3x3 stride-1 layers on the halo form too (two workgroups per CU)
        if (bn <= 64 && a.tune && a.tune->x6_halo_narrow && x6_halo_ok(a))
            return bn == 32 ? launch_x6_halo<32>(a, s) : launch_x6_halo<64>(a, s);
    }
    if (small) {
        if constexpr (TERMS == 2) {   // integer-valued canvases (face / plate stems): one A plane, two products
            if (bn == 32 && a.x_exact) return launch_x6<128, 32, 256, 1, 1>(a, s);
            if (bn == 64 && a.x_exact) return launch_x6<128, 64, 256, 1, 1>(a, s);
        }
        if (bn == 32) return launch_x6<128, 32, 256, 1, TERMS>(a, s);
        if (bn == 64) return launch_x6<128, 64, 256, 1, TERMS>(a, s);
        return launch_x6<128, 128, 256, 1, TERMS>(a, s);
    }
    if (bn == 32) return launch_x6<256, 32, 512, 2, TERMS>(a, s);
    if (bn == 64) return launch_x6<256, 64, 512, 2, TERMS>(a, s);
    if constexpr (TERMS == 2) {
        // short-K 1x1 layers (HBM-bound f32 tensors): a 128 x 128 two-stage tile at two
        // workgroups per CU, so one workgroup's epilogue / prologue overlaps the other's
        // main loop, and 4x the tiles of the 256 x 256 form balance the last round
        // (Cout 128 only: layer2 conv1 at K = 512 340 -> 305 us; the Cout 256 layers at
        // K = 512, FPN output1 / layer3.0 conv1, measured 7-13 % slower on it)
        if (a.tune && a.tune->x6_mid && a.kh == 1 && a.kw == 1 && a.kpad <= a.tune->x6_mid && a.cout == 128)
            return launch_x6<128, 128, 256, 2, TERMS>(a, s);
    }
    if constexpr (TERMS == 2) {   // 64 x 128 wave tiles: 2/3 of the LDS fragment reads per MFMA
        // (layer3/4 and FPN 12-20 % faster than 256 x 128; not below ~200 tiles: FPN output3,
        // 100 tiles, 137 -> 199 us)
        const long t256 = (long)((a.M + 255) / 256) * (a.cout / 256);
        if (a.tune && a.tune->x6_bn256 && a.cout % 256 == 0 && t256 >= 192) {
            if (x6_halo_ok(a)) return launch_x6_halo<256>(a, s);
            if (a.tune->x6_mf32) return launch_x6<256, 256, 512, 2, TERMS, 32>(a, s);
            return launch_x6_big<256, TERMS>(a, s);
        }
        // Cout 192 (the fused SSH conv5X5_1 + conv3X3): one 192-wide N tile instead of two
        // 128-wide ones with a quarter of the MFMAs on padding rows (level 0 1716 -> 1264 us,
        // level 1 526 -> 396; not for level 2's 100 tiles: 137 -> 178)
        if (a.tune && a.tune->x6_bn256 && a.cout == 192 && (a.M + 255) / 256 >= 192) {
            if (x6_halo_ok(a)) return launch_x6_halo<192>(a, s);
            return launch_x6_big<192, TERMS>(a, s);
        }
        // every eligible layer on the halo form whatever the batch (its K order differs);
        // option x6_halo_n64: Cout-128 layers with K <= x6_halo_n64 as two 64-wide N tiles,
        // two workgroups per CU (one's prologue / epilogue beside the other's main loop)
        if (x6_halo_ok(a)) {
            if (a.tune && a.cout == 128 && a.kpad <= a.tune->x6_halo_n64 && a.stride == 1) return launch_x6_halo<64>(a, s);
            return launch_x6_halo<128>(a, s);
        }
        if (a.tune && a.tune->x6_mf32) return launch_x6<256, 128, 512, 2, TERMS, 32>(a, s);
    }
    return launch_x6_big<128, TERMS>(a, s);
}

// fp16 pairs: bottleneck conv3 (1x1, K 64 / 128, ReLU) + downsample (1x1, K 64 / 256,
// strided, no activation) as conv1x1_x6_dual_kernel
bool vd_conv1x1_x6_dual_ok(const ConvArgs& a) {
    if (a.f32_split != 2 || !a.wx3 || !a.wx3_2 || !a.scale_x || !a.scale2_x) return false;
    if (a.kh != 1 || a.kw != 1 || a.pad != 0 || a.stride != 1 || a.kpad != a.cin_pad || a.kpad2 != a.cin2_pad) return false;
    if (a.act != VD_ACT_RELU || a.res_mode != VD_RES_NONE) return false;
    if (((a.ldx | a.xcoff | a.ldy | a.ycoff | a.ldx2 | a.xcoff2) & 7)) return false;
    // layer1.0 only: at layer2.0 (K 128 + 256) the weights of both fit LDS only as
    // 64-channel slices, every pixel is then split for 8 slices instead of 4 and the
    // pass measured level with the two launches (839 vs 424 + 433 us)
    return a.cin_pad == 64 && a.kpad2 == 64 && a.cout % 128 == 0;
}

hipError_t vd_launch_conv_x6(const ConvArgs& a0, hipStream_t s) {
    ConvArgs a = a0;
    a.dbg = a.tune ? (a.tune->x6_dbg & 3) | (a.tune->x6_one ? 4 : 0) | ((a.tune->x6_halo_dma & 3) << 3) |
                     (((a.tune->x6_dbg >> 2) & 15) << 5) | (a.tune->x6_tr_epi ? 0 : 512) |
                     (a.tune->x6_gemm_uni ? 0 : 1024) | (a.tune->x6_gemm_uni == 2 ? 2048 : 0) |
                     (a.tune->x6_halo_1b ? 0 : 4096) : 0;
    if (a.grp_co) {   // grouped: the halo form only, one 64-wide N tile per group
        if (a.grp_co != 64 || a.f32_split != 2 || !a.wx3 || !a.tune || !x6_halo_ok(a) || (a.ymax && a.B > kAmaxFrames))
            return hipErrorInvalidValue;
        a.scale = a.scale_x;
        return launch_x6_halo<64>(a, s);
    }
    if (a.x2) {
        if (!vd_conv1x1_x6_dual_ok(a) || (a.ymax && a.B > kAmaxFrames)) return hipErrorInvalidValue;
        return launch_dual_x6<2, 2, 8>(a, s);
    }
    if (a.f32_split == 2) {
        if (!a.scale_x || (a.ymax && a.B > kAmaxFrames)) return hipErrorInvalidValue;
        return launch_terms<2>(a, s);
    }
    ConvArgs b = a;
    b.xmax = nullptr;                                   // the bf16 triple needs no operand scaling
    return launch_terms<3>(b, s);
}

// Host: pack f32 weights [npad][kpad] (k = tap * cin_pad + c) into the split layout
// [npad][kpad / 32][3][32] bf16 (plane 0 = top 8 significand bits; same truncation
// split as the kernel's activations).
static inline unsigned f2u(float f) { unsigned u; std::memcpy(&u, &f, 4); return u; }
static inline float u2f(unsigned u) { float f; std::memcpy(&f, &u, 4); return f; }

void vd_pack_x6(const float* w, int npad, int kpad, uint16_t* out) {
    const int nk = kpad / KT;
    for (int n = 0; n < npad; ++n)
        for (int t = 0; t < nk; ++t)
            for (int k = 0; k < KT; ++k) {
                const float x = w[(size_t)n * kpad + t * KT + k];
                const unsigned u = f2u(x);
                const float r1 = x - u2f(u & 0xFFFF0000u);
                const unsigned v = f2u(r1);
                const float r2 = r1 - u2f(v & 0xFFFF0000u);
                uint16_t* o = out + (((size_t)n * nk + t) * 3) * KT + k;
                o[0] = (uint16_t)(u >> 16);
                o[KT] = (uint16_t)(v >> 16);
                o[2 * KT] = (uint16_t)(f2u(r2) >> 16);
            }
}

// Host: the fp16-pair layout [npad][kpad / 32][2][32] fp16 for f32_split = 2. Row n
// is scaled by 2^e[n] so its largest |w| lies in [2^14, 2^15) (hi = RNE(w 2^e),
// lo = RNE(w 2^e - hi)); row_inv[n] = 2^-e[n] is folded into the BN scale.
void vd_pack_x3h(const float* w, int npad, int kpad, uint16_t* out, float* row_inv) {
    const int nk = kpad / KT;
    for (int n = 0; n < npad; ++n) {
        float m = 0.f;
        for (int k = 0; k < kpad; ++k) m = std::max(m, std::fabs(w[(size_t)n * kpad + k]));
        int e = 0;
        if (m > 0.f) {
            (void)std::frexp(m, &e);
            e = std::min(100, std::max(-100, 15 - e));
        }
        row_inv[n] = std::ldexp(1.f, -e);
        for (int t = 0; t < nk; ++t)
            for (int k = 0; k < KT; ++k) {
                const float x = std::ldexp(w[(size_t)n * kpad + t * KT + k], e);
                const _Float16 h = (_Float16)x;
                const _Float16 l = (_Float16)(x - (float)h);
                uint16_t* o = out + (((size_t)n * nk + t) * 2) * KT + k;
                std::memcpy(o, &h, 2);
                std::memcpy(o + KT, &l, 2);
            }
    }
}
