// conv1x1.hip — streaming 1x1 convolution for the memory-bound layers of the
// forward (ResNet bottleneck conv1 / conv3 / downsample, K = Cin <= 256).
//
// Same arithmetic contract as conv.hip (bf16 operands, f32 accumulation, fused
// BN scale/shift + residual + activation), different schedule. Those layers move
// 3-5x more bytes than they compute for, so the block-synchronous GEMM — whose
// HBM traffic stops while a workgroup runs its epilogue — reaches only 2-3.7 TB/s.
// Here the weight slice (NCH output channels x K) is loaded into LDS once per
// workgroup, and every wave then streams groups of 16 output pixels on its own,
// with no workgroup barrier in the loop, so the waves of a CU interleave loads,
// MFMAs and stores freely and the memory pipe stays busy.
//
//   Per group: D^T[n][p] = sum_k W[n][k] * X[p][k]  (v_mfma_f32_16x16x32_bf16,
//   A operand = weight rows from LDS, B operand = 16 pixels' channels loaded
//   straight from the NHWC input as 16-B fragments). The transposed product puts
//   4 output channels of one pixel in each lane per 16x16 tile; the weight rows
//   are permuted in LDS so that tiles 2i and 2i+1 give a lane 8 CONSECUTIVE
//   channels (32i + 8q .. +8), and the epilogue stores 16 B (bf16) per lane
//   without an LDS pass, reading the residual in the same shape.
#include "vd_common.h"
#include <algorithm>
#include <cstdlib>

namespace {

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int lds_off(int row, int chunk) {
    return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4);
}

template <int ACT>
__device__ __forceinline__ float act_apply(float v, float slope) {
    if constexpr (ACT == VD_ACT_RELU) return v > 0.f ? v : 0.f;
    if constexpr (ACT == VD_ACT_LEAKY) return v > 0.f ? v : v * slope;
    if constexpr (ACT == VD_ACT_SILU) return v / (1.0f + __expf(-v));
    return v;
}


// KS: K / 32 (k-steps), NTT: 16-channel tiles per wave (NCH = 16 * NTT channels per
// workgroup), ACT / RES: activation and residual mode (compile-time: no per-element branches).
// TAPS: general KxK / strided / padded taps with any Cin (multiple of 8): each lane's
// 16-B fragment of k-step ks is (tap, 8 channels) = K elements (4ks + q)*8 .. +8 in the
// (kh, kw, c) order, gathered per pixel with zero padding (and zero past the last tap).
// KS2 > 0: DUAL — a second 1x1 conv (K2 = 32*KS2, weights w2, its own BN) over x2
// at stride2 is summed before the activation (bottleneck conv3 + downsample).
// F16: the fp16 plan (VD_PREC_FP16) on fp16 operands / activations, else bf16.
template <int KS, int NTT, int ACT, int RES, bool TAPS, int KS2, bool F16>
__global__ __launch_bounds__(512) void conv1x1_stream_kernel(ConvArgs a, int nchunks, int groups) {
    using HT = Half16<F16>;
    typedef typename HT::T T;
    constexpr int NCH = 16 * NTT;
    constexpr int KT = (KS + 1) / 2;                      // 128-byte K tiles per weight row
    constexpr int KT2 = (KS2 + 1) / 2;
    constexpr int WBYTES = KT * NCH * 128;
    constexpr int WBYTES2 = KT2 * NCH * 128;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* smem2 = smem + WBYTES;                          // second weight image (DUAL)
    float* s_scale = (float*)(smem + WBYTES + WBYTES2);
    float* s_shift = s_scale + NCH;
    float* s_scale2 = s_shift + NCH;
    float* s_shift2 = s_scale2 + NCH;

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int bid = blockIdx.x, xcd = bid & 7, local = bid >> 3;
    const int chunk = local % nchunks;                    // consecutive blocks of one XCD share pixels
    const int mblk = (local / nchunks) * 8 + xcd;
    const int nmblk = (gridDim.x / nchunks);              // grid = 8 * nchunks * k
    const int n0 = chunk * NCH;

    // weights [n0, n0+NCH) x [0, K) -> LDS image [kt][row][128 B] with the chunk swizzle;
    // LDS row 16j + i (tile j, MFMA row i) holds channel 32(j>>1) + 8(i>>2) + 4(j&1) + (i&3)
    {
        const T* w = (const T*)a.w;
        constexpr int CPR = KS * 4;                       // 16-B chunks per weight row (K/8)
        for (int i = tid; i < NCH * CPR; i += 512) {
            const int row = i / CPR, c = i - row * CPR;
            const int j = row >> 4, ii = row & 15;
            const int chn = NTT == 1 ? row : 32 * (j >> 1) + 8 * (ii >> 2) + 4 * (j & 1) + (ii & 3);
            const u32x4 v = *(const u32x4*)(w + (size_t)(n0 + chn) * a.kpad + c * 8);
            *(u32x4*)(smem + (c >> 3) * (NCH * 128) + lds_off(row, c & 7)) = v;
        }
        for (int i = tid; i < NCH; i += 512) {
            s_scale[i] = a.scale[n0 + i];
            s_shift[i] = a.shift[n0 + i];
        }
        if constexpr (KS2 > 0) {
            const T* w2 = (const T*)a.w2;
            constexpr int CPR2 = KS2 * 4;
            for (int i = tid; i < NCH * CPR2; i += 512) {
                const int row = i / CPR2, c = i - row * CPR2;
                const int j = row >> 4, ii = row & 15;
                const int chn = NTT == 1 ? row : 32 * (j >> 1) + 8 * (ii >> 2) + 4 * (j & 1) + (ii & 3);
                const u32x4 v = *(const u32x4*)(w2 + (size_t)(n0 + chn) * a.kpad2 + c * 8);
                *(u32x4*)(smem2 + (c >> 3) * (NCH * 128) + lds_off(row, c & 7)) = v;
            }
            for (int i = tid; i < NCH; i += 512) {
                s_scale2[i] = a.scale2[n0 + i];
                s_shift2[i] = a.shift2[n0 + i];
            }
        }
    }
    __syncthreads();

    const int p_lane = lane & 15, q = lane >> 4;          // pixel within group, channel quad / k chunk
    const int ohw = a.yh * a.yw;
    // TAPS: per-lane tap table (the lane's K chunk of every k-step is fixed)
    int toff[TAPS ? KS : 1], tdy[TAPS ? KS : 1], tdx[TAPS ? KS : 1];
    if constexpr (TAPS) {
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            const int ko = (ks * 4 + q) * 8;
            const int tap = ko / a.cin_pad, c = ko - tap * a.cin_pad;
            const int dy = tap / a.kw, dx = tap - dy * a.kw;
            const bool real = tap < a.kh * a.kw;
            toff[ks] = (dy * a.xw + dx) * a.ldx + c;
            tdy[ks] = real ? dy : -(1 << 20);               // past the last tap: always "outside"
            tdx[ks] = dx;
        }
    }
    const int wstride = nmblk * 8;
    constexpr int NR = NTT > 1 ? NTT / 2 : 1;
    // Load group G's input fragments into XF and its residual into RF.
#define VD_SLOAD(G, XF, RF, XF2)                                                               \
    do {                                                                                       \
        const int mu_ = (G) * 16 + p_lane;                                                     \
        const int m_ = mu_ < a.M ? mu_ : a.M - 1;   /* tail lanes load a valid pixel */        \
        const int b_ = m_ / ohw;                                                               \
        const int rem_ = m_ - b_ * ohw;                                                        \
        const int oy_ = rem_ / a.yw;                                                           \
        const int ox_ = rem_ - oy_ * a.yw;                                                     \
        if constexpr (TAPS) {                                                                  \
            const int iy0 = oy_ * a.stride - a.pad, ix0 = ox_ * a.stride - a.pad;              \
            const long base = (((long)b_ * a.xh + iy0) * a.xw + ix0) * a.ldx + a.xcoff;        \
            _Pragma("unroll") for (int ks = 0; ks < KS; ++ks) {                                \
                const int iy = iy0 + tdy[ks], ix = ix0 + tdx[ks];                              \
                const bool in = (unsigned)iy < (unsigned)a.xh && (unsigned)ix < (unsigned)a.xw;\
                const T* src = (const T*)a.x + (in ? base + toff[ks] : 0);                     \
                const u32x4 v = *(const u32x4*)src;                                            \
                XF[ks] = in ? v : u32x4{0u, 0u, 0u, 0u};                                       \
            }                                                                                  \
        } else {                                                                               \
            const T* xp = (const T*)a.x +                                                      \
                (((size_t)b_ * a.xh + oy_ * a.stride) * a.xw + ox_ * a.stride) * a.ldx + a.xcoff + q * 8; \
            _Pragma("unroll") for (int ks = 0; ks < KS; ++ks) XF[ks] = *(const u32x4*)(xp + ks * 32); \
        }                                                                                      \
        if constexpr (KS2 > 0) {                                                               \
            const T* xp2 = (const T*)a.x2 +                                                    \
                (((size_t)b_ * a.xh2 + oy_ * a.stride2) * a.xw2 + ox_ * a.stride2) * a.ldx2 + a.xcoff2 + q * 8; \
            _Pragma("unroll") for (int ks = 0; ks < (KS2 > 0 ? KS2 : 1); ++ks) XF2[ks] = *(const u32x4*)(xp2 + ks * 32); \
        }                                                                                      \
        if constexpr (RES != VD_RES_NONE) {                                                    \
            size_t roff;                                                                       \
            if (a.res_up) roff = ((size_t)(b_ * a.rh + (oy_ >> 1)) * a.rw + (ox_ >> 1)) * a.res_ld; \
            else roff = (size_t)m_ * a.res_ld;                                                 \
            if constexpr (NTT == 1) {                                                          \
                const unsigned* rp = (const unsigned*)((const T*)a.res + roff + a.res_coff + n0 + q * 4); \
                RF[0] = u32x4{rp[0], rp[1], 0u, 0u};                                           \
            } else {                                                                           \
                const T* rp = (const T*)a.res + roff + a.res_coff + n0 + q * 8;                \
                _Pragma("unroll") for (int i = 0; i < NR; ++i) RF[i] = *(const u32x4*)(rp + 32 * i); \
            }                                                                                  \
        }                                                                                      \
    } while (0)

    // Software-pipelined over the wave's groups: group g+1's loads are issued
    // before group g's MFMAs and stores, so every wave keeps reads in flight.
    constexpr int KX2 = KS2 > 0 ? KS2 : 1;
    u32x4 xf[KS], rf[NR], xf2[KX2];
    int g = mblk * 8 + wid;
    if (g < groups) VD_SLOAD(g, xf, rf, xf2);
    for (; g < groups; g += wstride) {
        // keep the weight-fragment LDS reads inside the loop (hoisting them all
        // would pin NTT*KS*4 VGPRs and cut the number of resident waves)
        asm volatile("" ::: "memory");
        u32x4 xn[KS], rn[NR], xn2[KX2];
        const int gn = g + wstride;
        if (gn < groups) VD_SLOAD(gn, xn, rn, xn2);
        const int mu = g * 16 + p_lane;
        const bool ok = mu < a.M;
        const int m = ok ? mu : a.M - 1;
        f32x4_t acc[NTT], acc2[KS2 > 0 ? NTT : 1];
#pragma unroll
        for (int j = 0; j < NTT; ++j) acc[j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
        if constexpr (KS2 > 0) {
#pragma unroll
            for (int j = 0; j < NTT; ++j) acc2[j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int ks = 0; ks < KS2; ++ks) {
                const char* wt = smem2 + (ks >> 1) * (NCH * 128);
                const int ch = (ks & 1) * 4 + q;
#pragma unroll
                for (int j = 0; j < NTT; ++j) {
                    const u32x4 wf = *(const u32x4*)(wt + lds_off(16 * j + p_lane, ch));
                    acc2[j] = HT::mfma(wf, xf2[ks], acc2[j]);
                }
            }
        }
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            const char* wt = smem + (ks >> 1) * (NCH * 128);
            const int ch = (ks & 1) * 4 + q;
#pragma unroll
            for (int j = 0; j < NTT; ++j) {
                const u32x4 wf = *(const u32x4*)(wt + lds_off(16 * j + p_lane, ch));
                acc[j] = HT::mfma(wf, xf[ks], acc[j]);
            }
        }
        if (ok) {
        if constexpr (NTT == 1) {   // lane holds channels n0 + 4q .. +4 of pixel m
            const size_t yo = (size_t)m * a.ldy + a.ycoff + n0 + q * 4;
            const float4 sc = *(const float4*)(s_scale + q * 4), sh = *(const float4*)(s_shift + q * 4);
            float v[4] = {acc[0][0] * sc.x + sh.x, acc[0][1] * sc.y + sh.y, acc[0][2] * sc.z + sh.z,
                          acc[0][3] * sc.w + sh.w};
            float rv[4] = {0.f, 0.f, 0.f, 0.f};
            if constexpr (RES != VD_RES_NONE) {
                rv[0] = HT::lo(rf[0][0]); rv[1] = HT::hi(rf[0][0]); rv[2] = HT::lo(rf[0][1]); rv[3] = HT::hi(rf[0][1]);
            }
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                float t = v[e];
                if constexpr (RES == VD_RES_PRE_ACT) t += rv[e];
                t = act_apply<ACT>(t, a.slope);
                if constexpr (RES == VD_RES_POST_ACT) t += rv[e];
                v[e] = t;
            }
            if (a.out_f32) {
                *(float4*)((float*)a.y + yo) = make_float4(v[0], v[1], v[2], v[3]);
            } else {
                typedef T t16x4_t __attribute__((ext_vector_type(4)));
                const t16x4_t o = {(T)v[0], (T)v[1], (T)v[2], (T)v[3]};
                *(t16x4_t*)((T*)a.y + yo) = o;
            }
        } else {
        // lane holds channels n0 + 32i + 8q + (0..3 from tile 2i, 4..7 from tile 2i+1) of pixel m
        const size_t yo = (size_t)m * a.ldy + a.ycoff + n0 + q * 8;
#pragma unroll
        for (int i = 0; i < NTT / 2; ++i) {
            const int c = 32 * i + q * 8;
            const float4 s0 = *(const float4*)(s_scale + c), s1 = *(const float4*)(s_scale + c + 4);
            const float4 h0 = *(const float4*)(s_shift + c), h1 = *(const float4*)(s_shift + c + 4);
            const f32x4_t& lo = acc[2 * i];
            const f32x4_t& hi = acc[2 * i + 1];
            float v[8] = {lo[0] * s0.x + h0.x, lo[1] * s0.y + h0.y, lo[2] * s0.z + h0.z, lo[3] * s0.w + h0.w,
                          hi[0] * s1.x + h1.x, hi[1] * s1.y + h1.y, hi[2] * s1.z + h1.z, hi[3] * s1.w + h1.w};
            if constexpr (KS2 > 0) {   // + bn(downsample): the branch sum, then the activation
                const float4 t0 = *(const float4*)(s_scale2 + c), t1 = *(const float4*)(s_scale2 + c + 4);
                const float4 g0 = *(const float4*)(s_shift2 + c), g1 = *(const float4*)(s_shift2 + c + 4);
                const f32x4_t& l2 = acc2[2 * i];
                const f32x4_t& h2 = acc2[2 * i + 1];
                const float u[8] = {l2[0] * t0.x + g0.x, l2[1] * t0.y + g0.y, l2[2] * t0.z + g0.z, l2[3] * t0.w + g0.w,
                                    h2[0] * t1.x + g1.x, h2[1] * t1.y + g1.y, h2[2] * t1.z + g1.z, h2[3] * t1.w + g1.w};
#pragma unroll
                for (int e = 0; e < 8; ++e) v[e] += u[e];
            }
            float rv[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
            if constexpr (RES != VD_RES_NONE) {
#pragma unroll
                for (int e = 0; e < 4; ++e) { rv[2 * e] = HT::lo(rf[i][e]); rv[2 * e + 1] = HT::hi(rf[i][e]); }
            }
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                float t = v[e];
                if constexpr (RES == VD_RES_PRE_ACT) t += rv[e];
                t = act_apply<ACT>(t, a.slope);
                if constexpr (RES == VD_RES_POST_ACT) t += rv[e];
                v[e] = t;
            }
            if (a.out_f32) {
                *(float4*)((float*)a.y + yo + 32 * i) = make_float4(v[0], v[1], v[2], v[3]);
                *(float4*)((float*)a.y + yo + 32 * i + 4) = make_float4(v[4], v[5], v[6], v[7]);
            } else {
                typename HT::V8 o;
#pragma unroll
                for (int e = 0; e < 8; ++e) o[e] = (T)v[e];
                *(typename HT::V8*)((T*)a.y + yo + 32 * i) = o;
            }
        }
        }
        }
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) xf[ks] = xn[ks];
#pragma unroll
        for (int i = 0; i < NR; ++i) rf[i] = rn[i];
        if constexpr (KS2 > 0) {
#pragma unroll
            for (int ks = 0; ks < KS2; ++ks) xf2[ks] = xn2[ks];
        }
    }
#undef VD_SLOAD
}

template <int KS, int NTT, int ACT, int RES, bool TAPS, int KS2, bool F16>
hipError_t launch_stream_t(const ConvArgs& a, hipStream_t s) {
    constexpr int NCH = 16 * NTT, KT = (KS + 1) / 2, KT2 = (KS2 + 1) / 2;
    constexpr size_t lds = (size_t)(KT + KT2) * NCH * 128 + 4 * NCH * sizeof(float);
    static const bool attr = [] {
        (void)hipFuncSetAttribute((const void*)conv1x1_stream_kernel<KS, NTT, ACT, RES, TAPS, KS2, F16>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        return true;
    }();
    (void)attr;
    // Persistent grid: as many workgroups as fit on the chip at once (each loads
    // its weight slice once), a multiple of 8 * nchunks for the XCD mapping.
    static const int resident = [] {
        int dev = 0, cus = 256, per_cu = 1;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, conv1x1_stream_kernel<KS, NTT, ACT, RES, TAPS, KS2, F16>,
                                                           512, lds);
        return std::max(1, cus * std::max(1, per_cu));
    }();
    const int nchunks = a.cout / NCH;
    const int groups = (a.M + 15) / 16;
    int k = std::max(1, resident / (8 * nchunks));
    k = std::min(k, std::max(1, (groups + 63) / 64));
    dim3 grid(8 * nchunks * k), block(512);
    hipLaunchKernelGGL((conv1x1_stream_kernel<KS, NTT, ACT, RES, TAPS, KS2, F16>), grid, block, lds, s, a, nchunks, groups);
    return hipGetLastError();
}

template <int KS, int NTT, int ACT, int RES, bool TAPS, int KS2 = 0>
hipError_t launch_stream(const ConvArgs& a, hipStream_t s) {
    return a.f16 ? launch_stream_t<KS, NTT, ACT, RES, TAPS, KS2, true>(a, s)
                 : launch_stream_t<KS, NTT, ACT, RES, TAPS, KS2, false>(a, s);
}

template <int KS, int NTT, bool TAPS>
hipError_t launch_mode(const ConvArgs& a, hipStream_t s) {
    if (a.act == VD_ACT_RELU) {
        if (a.res_mode == VD_RES_PRE_ACT) return launch_stream<KS, NTT, VD_ACT_RELU, VD_RES_PRE_ACT, TAPS>(a, s);
        if (a.res_mode == VD_RES_POST_ACT) return launch_stream<KS, NTT, VD_ACT_RELU, VD_RES_POST_ACT, TAPS>(a, s);
        return launch_stream<KS, NTT, VD_ACT_RELU, VD_RES_NONE, TAPS>(a, s);
    }
    if (a.act == VD_ACT_NONE) {
        if (a.res_mode == VD_RES_POST_ACT) return launch_stream<KS, NTT, VD_ACT_NONE, VD_RES_POST_ACT, TAPS>(a, s);
        if (a.res_mode == VD_RES_NONE) return launch_stream<KS, NTT, VD_ACT_NONE, VD_RES_NONE, TAPS>(a, s);
    }
    if (a.act == VD_ACT_SILU) {
        if (a.res_mode == VD_RES_POST_ACT) return launch_stream<KS, NTT, VD_ACT_SILU, VD_RES_POST_ACT, TAPS>(a, s);
        if (a.res_mode == VD_RES_NONE) return launch_stream<KS, NTT, VD_ACT_SILU, VD_RES_NONE, TAPS>(a, s);
    }
    return hipErrorInvalidValue;   // excluded by the eligibility checks
}

bool mode_ok(const ConvArgs& a) {
    return (a.act == VD_ACT_RELU) || (a.act == VD_ACT_NONE && a.res_mode != VD_RES_PRE_ACT) ||
           (a.act == VD_ACT_SILU && a.res_mode != VD_RES_PRE_ACT);
}

}  // namespace

// Eligible: bf16, 1x1 taps without padding, K in {64,128,256}, Cout a multiple of
// the channel slice, 16-B aligned channel offsets/strides for the residual and output.
bool vd_conv1x1_stream_ok(const ConvArgs& a) {
    if (!a.tune->conv_stream || a.kh != 1 || a.kw != 1 || a.pad != 0) return false;
    const bool k512 = a.cin_pad == 512 && a.tune->conv_stream512;
    if (a.cin_pad != 64 && a.cin_pad != 128 && a.cin_pad != 256 && !k512) return false;
    if (a.kpad < a.cin_pad || (a.cout % 64) != 0) return false;
    if ((a.ldx | a.xcoff) & 7) return false;
    if ((a.ldy | a.ycoff) & 7) return false;
    if (a.res_mode != VD_RES_NONE && ((a.res_ld | a.res_coff) & 7)) return false;
    return mode_ok(a);
}

// DUAL (conv3 + downsample): instantiated for ResNet layer1.0 (K 64 + 64) and
// layer2.0 (K 128 + 256 at stride 2), 128-channel slices, ReLU.
bool vd_conv1x1_dual_ok(const ConvArgs& a) {
    if (!a.x2 || (a.tune && !a.tune->conv_dual)) return false;
    if (a.kh != 1 || a.kw != 1 || a.pad != 0 || a.stride != 1 || a.act != VD_ACT_RELU || a.res_mode != VD_RES_NONE)
        return false;
    if (a.cout % 128 || a.kpad != a.cin_pad || a.kpad2 != a.cin2_pad) return false;
    if ((a.ldx | a.xcoff | a.ldy | a.ycoff | a.ldx2 | a.xcoff2) & 7) return false;
    return (a.cin_pad == 64 && a.cin2_pad == 64) || (a.cin_pad == 128 && a.cin2_pad == 256);
}

hipError_t vd_launch_conv1x1_stream(const ConvArgs& a, hipStream_t s) {
    if (a.x2) {
        if (a.cin_pad == 64) return launch_stream<2, 8, VD_ACT_RELU, VD_RES_NONE, false, 2>(a, s);
        return launch_stream<4, 8, VD_ACT_RELU, VD_RES_NONE, false, 8>(a, s);
    }
    // 256-channel slices at K 128/256 when Cout allows (bottleneck conv3 of layer2/3:
    // 1.1-1.2x the 128-channel form, tools/convbench k512; option stream_ntt=8 keeps 128),
    // else 128-channel slices (64 when Cout is not a multiple of 128)
    const int ntt_env = a.tune ? a.tune->stream_ntt : 16;
    if (ntt_env == 16 && a.cout % 256 == 0 && a.cin_pad == 128) return launch_mode<4, 16, false>(a, s);
    if (ntt_env == 16 && a.cout % 256 == 0 && a.cin_pad == 256) return launch_mode<8, 16, false>(a, s);
    const bool wide = a.cout % 128 == 0;
    if (a.cin_pad == 64) return wide ? launch_mode<2, 8, false>(a, s) : launch_mode<2, 4, false>(a, s);
    if (a.cin_pad == 128) return wide ? launch_mode<4, 8, false>(a, s) : launch_mode<4, 4, false>(a, s);
    if (a.cin_pad == 512) return wide ? launch_mode<16, 8, false>(a, s) : launch_mode<16, 4, false>(a, s);
    return wide ? launch_mode<8, 8, false>(a, s) : launch_mode<8, 4, false>(a, s);
}

// General taps (any kh x kw, stride, pad; Cin a multiple of 8) for small layers:
// K (padded to 64) <= TAPS_KMAX and Cout a multiple of 16 up to 128. Measured
// (tools/convbench yolo): 1.2-2.4x the implicit GEMM at K <= 288 (YOLO's 16-64
// channel layers), 0.6x at K = 576, hence the cut (option conv_taps=0 disables).
constexpr int TAPS_KMAX = 320;
bool vd_conv_taps_ok(const ConvArgs& a) {
    if (!a.tune->conv_taps) return false;
    if ((a.cin_pad & 7) || a.kpad > TAPS_KMAX || (a.kpad & 63) || (a.cout & 15) || a.cout > 128) return false;
    if ((a.ldx | a.xcoff) & 7) return false;
    const int align = (a.cout % 32 == 0) ? 7 : 3;        // 16-B (or 8-B for 16-channel slices) stores
    if ((a.ldy | a.ycoff) & align) return false;
    if (a.res_mode != VD_RES_NONE && ((a.res_ld | a.res_coff) & align)) return false;
    if (a.res_mode != VD_RES_NONE && a.res_up) return false;
    return mode_ok(a);
}

template <int KS>
hipError_t launch_taps_n(const ConvArgs& a, hipStream_t s) {
    // channel slice: 16 * NTT, largest that divides Cout with the slice weights <= 64 KB
    const int kb = a.kpad * 2;
    if (a.cout % 64 == 0 && 64 * kb <= 65536) return launch_mode<KS, 4, true>(a, s);
    if (a.cout % 32 == 0 && 32 * kb <= 65536) return launch_mode<KS, 2, true>(a, s);
    return launch_mode<KS, 1, true>(a, s);
}

hipError_t vd_launch_conv_taps(const ConvArgs& a, hipStream_t s) {
    switch (a.kpad / 32) {
        case 2: return launch_taps_n<2>(a, s);
        case 4: return launch_taps_n<4>(a, s);
        case 6: return launch_taps_n<6>(a, s);
        case 8: return launch_taps_n<8>(a, s);
        case 10: return launch_taps_n<10>(a, s);
        default: return hipErrorInvalidValue;
    }
}
