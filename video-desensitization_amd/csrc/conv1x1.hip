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

__device__ __forceinline__ float bf_lo(unsigned u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float bf_hi(unsigned u) { return __uint_as_float(u & 0xffff0000u); }

// KS: K / 32 (k-steps), NTT: 16-channel tiles per wave (NCH = 16 * NTT channels per
// workgroup), ACT / RES: activation and residual mode (compile-time: no per-element branches).
template <int KS, int NTT, int ACT, int RES>
__global__ __launch_bounds__(512) void conv1x1_stream_kernel(ConvArgs a, int nchunks, int groups) {
    constexpr int NCH = 16 * NTT;
    constexpr int KT = (KS + 1) / 2;                      // 128-byte K tiles per weight row
    constexpr int WBYTES = KT * NCH * 128;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    float* s_scale = (float*)(smem + WBYTES);
    float* s_shift = s_scale + NCH;

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int bid = blockIdx.x, xcd = bid & 7, local = bid >> 3;
    const int chunk = local % nchunks;                    // consecutive blocks of one XCD share pixels
    const int mblk = (local / nchunks) * 8 + xcd;
    const int nmblk = (gridDim.x / nchunks);              // grid = 8 * nchunks * k
    const int n0 = chunk * NCH;

    // weights [n0, n0+NCH) x [0, K) -> LDS image [kt][row][128 B] with the chunk swizzle;
    // LDS row 16j + i (tile j, MFMA row i) holds channel 32(j>>1) + 8(i>>2) + 4(j&1) + (i&3)
    {
        const __bf16* w = (const __bf16*)a.w;
        constexpr int CPR = KS * 4;                       // 16-B chunks per weight row (K/8)
        for (int i = tid; i < NCH * CPR; i += 512) {
            const int row = i / CPR, c = i - row * CPR;
            const int j = row >> 4, ii = row & 15;
            const int chn = 32 * (j >> 1) + 8 * (ii >> 2) + 4 * (j & 1) + (ii & 3);
            const u32x4 v = *(const u32x4*)(w + (size_t)(n0 + chn) * a.kpad + c * 8);
            *(u32x4*)(smem + (c >> 3) * (NCH * 128) + lds_off(row, c & 7)) = v;
        }
        for (int i = tid; i < NCH; i += 512) {
            s_scale[i] = a.scale[n0 + i];
            s_shift[i] = a.shift[n0 + i];
        }
    }
    __syncthreads();

    const int p_lane = lane & 15, q = lane >> 4;          // pixel within group, channel quad / k chunk
    const int ohw = a.yh * a.yw;
    const int wstride = nmblk * 8;
    for (int g = mblk * 8 + wid; g < groups; g += wstride) {
        // keep the weight-fragment LDS reads inside the loop (hoisting them all
        // would pin NTT*KS*4 VGPRs and cut the number of resident waves)
        asm volatile("" ::: "memory");
        const int mu = g * 16 + p_lane;
        const bool ok = mu < a.M;
        const int m = ok ? mu : a.M - 1;          // tail lanes load a valid pixel, store nothing
        const int b = m / ohw;
        const int rem = m - b * ohw;
        const int oy = rem / a.yw;
        const int ox = rem - oy * a.yw;
        // input fragments: pixel p_lane, channels ks*32 + 8q .. +8
        const __bf16* xp = (const __bf16*)a.x +
                           (((size_t)b * a.xh + oy * a.stride) * a.xw + ox * a.stride) * a.ldx + a.xcoff + q * 8;
        u32x4 xf[KS];
#pragma unroll
        for (int ks = 0; ks < KS; ++ks)
            xf[ks] = *(const u32x4*)(xp + ks * 32);
        // residual: pixel p_lane, channels n0 + 32i + 8q .. +8 (16 B each)
        u32x4 rf[NTT / 2];
        if constexpr (RES != VD_RES_NONE) {
            size_t roff;
            if (a.res_up) roff = ((size_t)(b * a.rh + (oy >> 1)) * a.rw + (ox >> 1)) * a.res_ld;
            else roff = (size_t)m * a.res_ld;
            const __bf16* rp = (const __bf16*)a.res + roff + a.res_coff + n0 + q * 8;
#pragma unroll
            for (int i = 0; i < NTT / 2; ++i) rf[i] = *(const u32x4*)(rp + 32 * i);
        }
        f32x4_t acc[NTT];
#pragma unroll
        for (int j = 0; j < NTT; ++j) acc[j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            const char* wt = smem + (ks >> 1) * (NCH * 128);
            const int ch = (ks & 1) * 4 + q;
#pragma unroll
            for (int j = 0; j < NTT; ++j) {
                const u32x4 wf = *(const u32x4*)(wt + lds_off(16 * j + p_lane, ch));
                acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, wf),
                                                                 __builtin_bit_cast(bf16x8_t, xf[ks]), acc[j], 0, 0, 0);
            }
        }
        // lane holds channels n0 + 32i + 8q + (0..3 from tile 2i, 4..7 from tile 2i+1) of pixel m
        if (!ok) continue;
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
            float rv[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
            if constexpr (RES != VD_RES_NONE) {
#pragma unroll
                for (int e = 0; e < 4; ++e) { rv[2 * e] = bf_lo(rf[i][e]); rv[2 * e + 1] = bf_hi(rf[i][e]); }
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
                bf16x8_t o;
#pragma unroll
                for (int e = 0; e < 8; ++e) o[e] = (__bf16)v[e];
                *(bf16x8_t*)((__bf16*)a.y + yo + 32 * i) = o;
            }
        }
    }
}

template <int KS, int NTT, int ACT, int RES>
hipError_t launch_stream(const ConvArgs& a, hipStream_t s) {
    constexpr int NCH = 16 * NTT, KT = (KS + 1) / 2;
    constexpr size_t lds = (size_t)KT * NCH * 128 + 2 * NCH * sizeof(float);
    static const bool attr = [] {
        (void)hipFuncSetAttribute((const void*)conv1x1_stream_kernel<KS, NTT, ACT, RES>,
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
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, conv1x1_stream_kernel<KS, NTT, ACT, RES>, 512, lds);
        return std::max(1, cus * std::max(1, per_cu));
    }();
    const int nchunks = a.cout / NCH;
    const int groups = (a.M + 15) / 16;
    int k = std::max(1, resident / (8 * nchunks));
    k = std::min(k, std::max(1, (groups + 63) / 64));
    dim3 grid(8 * nchunks * k), block(512);
    hipLaunchKernelGGL((conv1x1_stream_kernel<KS, NTT, ACT, RES>), grid, block, lds, s, a, nchunks, groups);
    return hipGetLastError();
}

template <int KS, int NTT>
hipError_t launch_mode(const ConvArgs& a, hipStream_t s) {
    if (a.act == VD_ACT_RELU) {
        if (a.res_mode == VD_RES_PRE_ACT) return launch_stream<KS, NTT, VD_ACT_RELU, VD_RES_PRE_ACT>(a, s);
        if (a.res_mode == VD_RES_POST_ACT) return launch_stream<KS, NTT, VD_ACT_RELU, VD_RES_POST_ACT>(a, s);
        return launch_stream<KS, NTT, VD_ACT_RELU, VD_RES_NONE>(a, s);
    }
    if (a.act == VD_ACT_NONE) {
        if (a.res_mode == VD_RES_POST_ACT) return launch_stream<KS, NTT, VD_ACT_NONE, VD_RES_POST_ACT>(a, s);
        if (a.res_mode == VD_RES_NONE) return launch_stream<KS, NTT, VD_ACT_NONE, VD_RES_NONE>(a, s);
    }
    if (a.act == VD_ACT_SILU && a.res_mode == VD_RES_NONE) return launch_stream<KS, NTT, VD_ACT_SILU, VD_RES_NONE>(a, s);
    return hipErrorInvalidValue;   // excluded by vd_conv1x1_stream_ok
}

}  // namespace

// Eligible: bf16, 1x1 taps without padding, K in {64,128,256}, Cout a multiple of
// the channel slice, 16-B aligned channel offsets/strides for the residual and output.
bool vd_conv1x1_stream_ok(const ConvArgs& a) {
    static const bool on = [] { const char* e = getenv("VD_CONV_STREAM"); return !e || atoi(e) != 0; }();
    if (!on || a.kh != 1 || a.kw != 1 || a.pad != 0) return false;
    if (a.cin_pad != 64 && a.cin_pad != 128 && a.cin_pad != 256) return false;
    if (a.kpad < a.cin_pad || (a.cout % 64) != 0) return false;
    if ((a.ldx | a.xcoff) & 7) return false;
    if ((a.ldy | a.ycoff) & 7) return false;
    if (a.res_mode != VD_RES_NONE && ((a.res_ld | a.res_coff) & 7)) return false;
    const bool mode_ok = (a.act == VD_ACT_RELU) ||
                         (a.act == VD_ACT_NONE && a.res_mode != VD_RES_PRE_ACT) ||
                         (a.act == VD_ACT_SILU && a.res_mode == VD_RES_NONE);
    return mode_ok;
}

hipError_t vd_launch_conv1x1_stream(const ConvArgs& a, hipStream_t s) {
    // 128-channel slices (64 when Cout is not a multiple of 128); K 64/128/256
    const bool wide = a.cout % 128 == 0;
    if (a.cin_pad == 64) return wide ? launch_mode<2, 8>(a, s) : launch_mode<2, 4>(a, s);
    if (a.cin_pad == 128) return wide ? launch_mode<4, 8>(a, s) : launch_mode<4, 4>(a, s);
    return wide ? launch_mode<8, 8>(a, s) : launch_mode<8, 4>(a, s);
}
