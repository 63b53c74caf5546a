// stem.hip — the ResNet-50 stem of RetinaFace in one kernel: conv1 7x7/2 + bn1 +
// relu, then maxpool 3x3/2 pad 1 (torchvision resnet50 [ext] as loaded from the
// reference's body.conv1 / body.bn1 / body.maxpool, detect_face/retinaface.py:53-60).
//
// The conv runs in its space-to-depth form (face_net.cpp stem_s2d: a 4x4 stride-1
// pad-1 conv over X'[Y][X][16] = the letterboxed canvas in 2x2 sub-pixel blocks),
// the same bf16 products and K order as the streaming taps kernel, so the stem
// activations are identical; they are rounded to bf16 and pooled in LDS, and only
// the pooled map (1/4 of the stem's bytes) reaches HBM -- the 64x320x320x64 stem
// map of a 640x640 batch (839 MB at B = 64) is never written or read back.
//
// Persistent workgroups of 4 waves walk 8x8 tiles of pool outputs:
//   - the 20x20 X' tile (13 KB) arrives by LDS-DMA; the next tile's is issued as
//     soon as stage A is done with the buffer (or, double-buffered, at the top);
//   - stage A: the 17x17 stem outputs under the pool windows (19 groups of 16
//     pixels) as D^T = W . X^T with v_mfma_f32_16x16x32_bf16; wave w holds the
//     weight fragments of channels 32(w&1) .. +32 in VGPRs for good and takes every
//     other group; BN + ReLU, bf16, 16-B LDS writes of 8 consecutive channels;
//   - stage B: the 3x3/2 max of 64 pool pixels x 8 channel chunks (bf16 values >= 0
//     after the ReLU compare as their bit patterns; zero padding = the -inf padding
//     of the pool over non-negative inputs), 16-B stores.
#include "vd_common.h"

#include <cstdlib>

namespace {

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void_t;

constexpr int PT = 8;                     // pool tile (PT x PT outputs)
constexpr int SE = 2 * PT + 1;            // stem tile edge (17)
constexpr int SP = SE * SE;               // 289 stem pixels
constexpr int NG = (SP + 15) / 16;        // 19 groups of 16
constexpr int XE = SE + 3;                // X' tile edge (20): 4x4 taps, pad 1
constexpr int XP = XE * XE;               // 400 X' pixels x 32 B
constexpr int NDMA = (XP * 32 + 1023) / 1024;
constexpr int DPW = (NDMA + 3) / 4;       // DMA instructions per wave (padded, see block.hip)
constexpr int XBUF = NDMA * 1024;
constexpr int STB = NG * 16 * 128;        // stem tile image: 304 rows x 64 channels bf16
constexpr int VMCNT2 = 0x0F72;            // s_waitcnt vmcnt(2) (expcnt / lgkmcnt: no wait)

__device__ __forceinline__ int st_off(int row, int chunk) {
    return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4);
}

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

// max of two pairs of non-negative bf16 -- or fp16: both formats' non-negative bit
// patterns order as unsigned 16-bit integers: one v_pk_max_u16
__device__ __forceinline__ unsigned max_bf16x2(unsigned a, unsigned b) {
    return __builtin_bit_cast(unsigned, __builtin_elementwise_max(__builtin_bit_cast(u16x2, a),
                                                                 __builtin_bit_cast(u16x2, b)));
}

// NXB: X' tile buffers (2 = next tile's DMA overlaps this tile, 1 = more workgroups per
// CU); F16: the fp16 plan (VD_PREC_FP16: fp16 canvas, weights and pooled map)
template <int NXB, bool F16>
__global__ __launch_bounds__(256, 2) void stem_pool_kernel(StemPoolArgs a) {
    using HT = Half16<F16>;
    typedef typename HT::T E16;
    const auto mfma = [](const u32x4& x, const u32x4& y, const f32x4_t& c) { return HT::mfma(x, y, c); };
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* lx = smem;                       // NXB x XBUF
    char* lst = smem + NXB * XBUF;         // STB
    char* lscratch = lst + STB;            // 1 KB sink of the padding DMA slots

    const int tid = threadIdx.x, lane = tid & 63, li0 = lane & 15, g0 = lane >> 4;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int np = w & 1, gh = w >> 1;
    const int SH = a.xh - 1, SW = a.xw - 1;                   // stem output (4x4, pad 1)
    const int tpr = (a.ph + PT - 1) / PT, tpc = (a.pw + PT - 1) / PT, tpf = tpr * tpc;
    const int T = a.B * tpf;
    const int G = gridDim.x, bid = blockIdx.x;
    int t0, tstep, tend;
    if (G >= 8) {   // XCD-contiguous tile ranges
        const int x8 = bid & 7;
        t0 = (int)((long)x8 * T / 8) + (bid >> 3);
        tstep = G / 8 + (x8 < G % 8 ? 1 : 0);
        tend = (int)((long)(x8 + 1) * T / 8);
    } else {
        t0 = bid; tstep = G; tend = T;
    }
    if (t0 >= tend) return;
    const size_t fx = (size_t)a.xh * a.xw * 16;              // X' elements per frame

    auto issue_x = [&](int t, int buf) {
        const int b = t / tpf, r0 = t - b * tpf;
        const int ty = r0 / tpc, tx = r0 - ty * tpc;
        const int xr0 = 2 * PT * ty - 2, xc0 = 2 * PT * tx - 2;   // X' origin of the tile
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            (void*)((const E16*)a.x + (size_t)b * fx), 0, (int)(fx * 2), 0x00020000);
        char* dst = lx + buf * XBUF;
#pragma unroll
        for (int k = 0; k < DPW; ++k) {
            const int i = w + 4 * k;
            const bool real = i < NDMA;
            const int xp = 32 * i + (lane >> 1), ch = lane & 1;
            const int xr = xp / XE, xc = xp - xr * XE;
            const int iy = xr0 + xr, ix = xc0 + xc;
            const bool in = real && xp < XP && (unsigned)iy < (unsigned)a.xh && (unsigned)ix < (unsigned)a.xw;
            const unsigned off = in ? (unsigned)(((iy * a.xw + ix) * 16 + ch * 8) * 2) : 0x80000000u;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void_t*)(real ? dst + i * 1024 : lscratch), 16, off, 0, 0,
                                                     0);
        }
    };
    issue_x(t0, 0);

    // stationary: weight fragments of this wave's 32 channels (2 tiles x 8 k-steps) and BN
    const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc((void*)a.wf, 0, 0x7fffffff, 0x00020000);
    u32x4 wf[2][8];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int s = 0; s < 8; ++s)
            wf[j][s] = __builtin_amdgcn_raw_buffer_load_b128(rw, (unsigned)lane * 16u, ((2 * np + j) * 8 + s) * 1024, 0);
    float sc[8], sh[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        sc[e] = a.scale[32 * np + 8 * g0 + e];
        sh[e] = a.shift[32 * np + 8 * g0 + e];
    }

    int buf = 0;
#pragma unroll 1
    for (int t = t0; t < tend; t += tstep) {
        const int b = t / tpf, r0 = t - b * tpf;
        const int ty = r0 / tpc, tx = r0 - ty * tpc;
        const int sy0 = 2 * PT * ty - 1, sx0 = 2 * PT * tx - 1;   // stem origin of the tile
        const char* lxc = lx + buf * XBUF;
        // this tile's X' (DMA): vmcnt counts loads, stores and LDS-DMA together in issue
        // order, and the previous tile's 2 stores per thread are the only younger ops
        __builtin_amdgcn_s_waitcnt(VMCNT2);
        __syncthreads();
        if (NXB == 2 && t + tstep < tend) issue_x(t + tstep, buf ^ 1);   // no register loads follow
        int li = li0, g = g0;
        asm volatile("" : "+v"(li), "+v"(g));

        // ---- stage A: stem outputs of this wave's groups, channels 32np .. +32 ----
#pragma unroll 1
        for (int G16 = gh; G16 < NG; G16 += 2) {
            const int p = 16 * G16 + li;
            const int r = p / SE, c = p - r * SE;
            f32x4_t acc[2] = {f32x4_t{0.f, 0.f, 0.f, 0.f}, f32x4_t{0.f, 0.f, 0.f, 0.f}};
            u32x4 xf[8];
#pragma unroll
            for (int s = 0; s < 8; ++s) {
                const int tap = 2 * s + (g >> 1), ta = tap >> 2, tb = tap & 3;
                xf[s] = *(const u32x4*)(lxc + ((r + ta) * XE + c + tb) * 32 + (g & 1) * 16);
            }
#pragma unroll
            for (int s = 0; s < 8; ++s) {
                acc[0] = mfma(wf[0][s], xf[s], acc[0]);
                acc[1] = mfma(wf[1][s], xf[s], acc[1]);
            }
            const int sy = sy0 + r, sx = sx0 + c;
            const bool in = p < SP && (unsigned)sy < (unsigned)SH && (unsigned)sx < (unsigned)SW;
            typename HT::V8 o;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const float v = acc[e >> 2][e & 3] * sc[e] + sh[e];
                o[e] = (E16)(in && v > 0.f ? v : 0.f);
            }
            *(typename HT::V8*)(lst + st_off(p, 4 * np + g)) = o;
        }
        __syncthreads();
        if (NXB == 1 && t + tstep < tend) issue_x(t + tstep, 0);   // X' buffer free once stage A is done

        // ---- stage B: 3x3/2 max pool of the tile, 8 channels per thread ----
        {
            // stores through a descriptor, unconditional (past the frame: out-of-range
            // offset, dropped) so every thread issues exactly 2 per tile (see vmcnt above)
            const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc(
                (void*)((E16*)a.y + (size_t)b * a.ph * a.pw * 64), 0, (int)((size_t)a.ph * a.pw * 128), 0x00020000);
#pragma unroll
            for (int pass = 0; pass < 2; ++pass) {
                const int q = pass * 32 + (tid >> 3), ch = tid & 7;
                const int pi = q >> 3, pj = q & 7;
                u32x4 m = {0u, 0u, 0u, 0u};
#pragma unroll
                for (int dy = 0; dy < 3; ++dy)
#pragma unroll
                    for (int dx = 0; dx < 3; ++dx) {
                        const u32x4 v = *(const u32x4*)(lst + st_off((2 * pi + dy) * SE + 2 * pj + dx, ch));
#pragma unroll
                        for (int e = 0; e < 4; ++e) m[e] = max_bf16x2(m[e], v[e]);
                    }
                const int py = PT * ty + pi, px = PT * tx + pj;
                const unsigned off = py < a.ph && px < a.pw ? (unsigned)(((py * a.pw + px) * 64 + 8 * ch) * 2) : 0x80000000u;
                __builtin_amdgcn_raw_buffer_store_b128(m, ry, off, 0, 0);
            }
        }
        if (NXB == 2) buf ^= 1;
    }
}

template <int NXB, bool F16>
hipError_t launch_stem(const StemPoolArgs& a, hipStream_t s) {
    constexpr size_t lds = NXB * XBUF + STB + 1024;
    static const int cus = [] {
        (void)hipFuncSetAttribute((const void*)stem_pool_kernel<NXB, F16>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)lds);
        int dev = 0, n = 256;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
        return n > 0 ? n : 256;
    }();
    const int per_cu = NXB == 2 ? 2 : 3;                 // LDS: 66 KB / 53 KB per workgroup
    const int tiles = a.B * ((a.ph + PT - 1) / PT) * ((a.pw + PT - 1) / PT);
    const int grid = tiles < per_cu * cus ? tiles : per_cu * cus;   // persistent
    hipLaunchKernelGGL((stem_pool_kernel<NXB, F16>), dim3(grid), dim3(256), lds, s, a);
    return hipGetLastError();
}

}  // namespace

bool vd_stem_pool_ok(int xh, int xw, int ph, int pw) {
    const int sh = xh - 1, sw = xw - 1;
    return xh >= 2 && xw >= 2 && ph == (sh - 1) / 2 + 1 && pw == (sw - 1) / 2 + 1 &&
           (double)xh * xw * 16 * 2 < 2147483647.0 && (double)ph * pw * 128 < 2147483647.0;
}

hipError_t vd_launch_stem_pool(const StemPoolArgs& a, hipStream_t s) {
    if (a.B <= 0) return hipSuccess;
    // one X' buffer and three workgroups per CU measured 9 % faster than two buffers
    // (DMA overlapping the whole tile) at two workgroups per CU: the kernel is
    // latency-bound, occupancy wins
    return a.f16 ? launch_stem<1, true>(a, s) : launch_stem<1, false>(a, s);
}

// ---------------------------------------------------------------------------
// fp32 plan (fp16 pairs): the same fused stem + pool. X' is the fp16 canvas (its
// values, pixel - mean, are integers: exact), the weights are the conv's fp16 pair
// (hi, lo; per-channel power-of-two scale folded into the BN scale), so each MAC is
// two f16 products with f32 accumulation (v_mfma_f32_16x16x32_f16, small term
// first). The stem tile lives in LDS as f32 (64 channels x 4 B per pixel), so pool
// tiles are 6x6 (13x13 stem pixels, 54 KB per workgroup, two per CU); the pooled
// map is f32 and its per-frame max |y| goes to a.ymax for layer1's operand scale.
namespace {

constexpr int PT3 = 6;                     // pool tile
constexpr int SE3 = 2 * PT3 + 1;           // 13
constexpr int SP3 = SE3 * SE3;             // 169 stem pixels
constexpr int NG3 = (SP3 + 15) / 16;       // 11 groups of 16
constexpr int XE3 = SE3 + 3;               // 16
constexpr int XP3 = XE3 * XE3;             // 256 X' pixels x 32 B
constexpr int NDMA3 = (XP3 * 32 + 1023) / 1024;
constexpr int DPW3 = (NDMA3 + 3) / 4;
constexpr int XBUF3 = NDMA3 * 1024;
constexpr int STB3 = NG3 * 16 * 256;       // 176 rows x 64 channels f32
constexpr int VMCNT4 = 0x0F74;             // s_waitcnt vmcnt(4)

// chunk: 16 B = 4 channels, 0..15. Key x ^ bit1(x) of x = row & 15: 16 consecutive
// rows (stage A's 16 lanes) get 16 distinct keys, and rows r, r + 2 (stage B's two
// pool pixels per 16 lanes) keys of opposite parity, so their even chunks don't collide
__device__ __forceinline__ int st_off3(int row, int chunk) {
    return row * 256 + ((chunk ^ (row & 15) ^ ((row >> 1) & 1)) << 4);
}

__device__ __forceinline__ f32x4_t mfma16(const u32x4& a, const u32x4& b, const f32x4_t& c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8_t, a), __builtin_bit_cast(f16x8_t, b), c, 0,
                                                  0, 0);
}

__global__ __launch_bounds__(256, 2) void stem_pool32_kernel(StemPoolArgs a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* lx = smem;                       // 2 x XBUF3: X' of this tile and the next
    char* lst = smem + 2 * XBUF3;          // STB3
    char* lscratch = lst + STB3;           // 1 KB sink of the padding DMA slots
    unsigned* s_amax = (unsigned*)(lscratch + 1024);

    const int tid = threadIdx.x, lane = tid & 63, li0 = lane & 15, g0 = lane >> 4;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int np = w & 1, gh = w >> 1;
    const int SH = a.xh - 1, SW = a.xw - 1;
    const int tpr = (a.ph + PT3 - 1) / PT3, tpc = (a.pw + PT3 - 1) / PT3, tpf = tpr * tpc;
    const int T = a.B * tpf;
    const int G = gridDim.x, bid = blockIdx.x;
    int t0, tstep, tend;
    if (G >= 8) {
        const int x8 = bid & 7;
        t0 = (int)((long)x8 * T / 8) + (bid >> 3);
        tstep = G / 8 + (x8 < G % 8 ? 1 : 0);
        tend = (int)((long)(x8 + 1) * T / 8);
    } else {
        t0 = bid; tstep = G; tend = T;
    }
    for (int f = tid; f < a.B; f += 256) s_amax[f] = 0u;
    const size_t fx = (size_t)a.xh * a.xw * 16;

    auto issue_x = [&](int t, int buf) {
        const int b = t / tpf, r0 = t - b * tpf;
        const int ty = r0 / tpc, tx = r0 - ty * tpc;
        const int xr0 = 2 * PT3 * ty - 2, xc0 = 2 * PT3 * tx - 2;
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            (void*)((const _Float16*)a.x + (size_t)b * fx), 0, (int)(fx * 2), 0x00020000);
#pragma unroll
        for (int k = 0; k < DPW3; ++k) {
            const int i = w + 4 * k;
            const bool real = i < NDMA3;
            const int xp = 32 * i + (lane >> 1), ch = lane & 1;
            const int xr = xp / XE3, xc = xp - xr * XE3;
            const int iy = xr0 + xr, ix = xc0 + xc;
            const bool in = real && xp < XP3 && (unsigned)iy < (unsigned)a.xh && (unsigned)ix < (unsigned)a.xw;
            const unsigned off = in ? (unsigned)(((iy * a.xw + ix) * 16 + ch * 8) * 2) : 0x80000000u;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void_t*)(real ? lx + buf * XBUF3 + i * 1024 : lscratch), 16,
                                                     off, 0, 0, 0);
        }
    };
    if (t0 < tend) issue_x(t0, 0);

    // stationary: hi / lo weight fragments of this wave's 32 channels and the BN terms
    const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc((void*)a.wf, 0, 0x7fffffff, 0x00020000);
    u32x4 wh[2][8], wl[2][8];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int s = 0; s < 8; ++s) {
            wh[j][s] = __builtin_amdgcn_raw_buffer_load_b128(rw, (unsigned)lane * 16u, ((2 * np + j) * 8 + s) * 1024, 0);
            wl[j][s] = __builtin_amdgcn_raw_buffer_load_b128(rw, (unsigned)lane * 16u,
                                                             32 * 1024 + ((2 * np + j) * 8 + s) * 1024, 0);
        }
    float sc[8], sh[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        sc[e] = a.scale[32 * np + 8 * g0 + e];
        sh[e] = a.shift[32 * np + 8 * g0 + e];
    }

    int xb = 0;                            // X' buffer of this tile
#pragma unroll 1
    for (int t = t0; t < tend; t += tstep, xb ^= 1) {
        const int b = t / tpf, r0 = t - b * tpf;
        const int ty = r0 / tpc, tx = r0 - ty * tpc;
        const int sy0 = 2 * PT3 * ty - 1, sx0 = 2 * PT3 * tx - 1;
        // this tile's X' (DMA, issued a whole tile ago); the previous tile's 4 stores per
        // thread are the only younger ops
        __builtin_amdgcn_s_waitcnt(VMCNT4);
        __syncthreads();
        // the next tile's X' into the other buffer (stage A of the previous tile, its
        // last reader, finished before the barrier above)
        if (t + tstep < tend) issue_x(t + tstep, xb ^ 1);
        const char* lxt = lx + xb * XBUF3;
        int li = li0, g = g0;
        asm volatile("" : "+v"(li), "+v"(g));

        // ---- stage A: stem outputs of this wave's groups, channels 32np .. +32 ----
#pragma unroll 1
        for (int G16 = gh; G16 < NG3; G16 += 2) {
            const int p = 16 * G16 + li;
            const int r = p / SE3, c = p - r * SE3;
            f32x4_t acc[2] = {f32x4_t{0.f, 0.f, 0.f, 0.f}, f32x4_t{0.f, 0.f, 0.f, 0.f}};
            u32x4 xf[8];
#pragma unroll
            for (int s = 0; s < 8; ++s) {
                const int tap = 2 * s + (g >> 1), ta = tap >> 2, tb = tap & 3;
                const int rr = r + ta < XE3 ? r + ta : XE3 - 1;   // rows past the tile (p >= SP3): any X'
                xf[s] = *(const u32x4*)(lxt + (rr * XE3 + (c + tb < XE3 ? c + tb : XE3 - 1)) * 32 + (g & 1) * 16);
            }
#pragma unroll
            for (int s = 0; s < 8; ++s) {
                acc[0] = mfma16(wl[0][s], xf[s], acc[0]);
                acc[1] = mfma16(wl[1][s], xf[s], acc[1]);
                acc[0] = mfma16(wh[0][s], xf[s], acc[0]);
                acc[1] = mfma16(wh[1][s], xf[s], acc[1]);
            }
            const int sy = sy0 + r, sx = sx0 + c;
            const bool in = p < SP3 && (unsigned)sy < (unsigned)SH && (unsigned)sx < (unsigned)SW;
            float o[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const float v = acc[e >> 2][e & 3] * sc[e] + sh[e];
                o[e] = in && v > 0.f ? v : 0.f;
            }
            const int cg = 2 * (4 * np + g);
            *(float4*)(lst + st_off3(p, cg)) = make_float4(o[0], o[1], o[2], o[3]);
            *(float4*)(lst + st_off3(p, cg + 1)) = make_float4(o[4], o[5], o[6], o[7]);
        }
        __syncthreads();

        // ---- stage B: 3x3/2 max pool of the tile, 8 channels per item, 2 items per thread ----
        {
            const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc(
                (void*)((float*)a.y + (size_t)b * a.ph * a.pw * 64), 0, (int)((size_t)a.ph * a.pw * 256), 0x00020000);
            float tm = 0.f;
#pragma unroll
            for (int pass = 0; pass < 2; ++pass) {
                const int it = pass * 256 + tid;
                const int q = it >> 3, ch = it & 7;
                const bool item = q < PT3 * PT3;
                const int qq = item ? q : 0;
                const int pi = qq / PT3, pj = qq - pi * PT3;
                float4 m0 = make_float4(0.f, 0.f, 0.f, 0.f), m1 = m0;
#pragma unroll
                for (int dy = 0; dy < 3; ++dy)
#pragma unroll
                    for (int dx = 0; dx < 3; ++dx) {
                        const int row = (2 * pi + dy) * SE3 + 2 * pj + dx;
                        const float4 v0 = *(const float4*)(lst + st_off3(row, 2 * ch));
                        const float4 v1 = *(const float4*)(lst + st_off3(row, 2 * ch + 1));
                        m0.x = fmaxf(m0.x, v0.x); m0.y = fmaxf(m0.y, v0.y); m0.z = fmaxf(m0.z, v0.z); m0.w = fmaxf(m0.w, v0.w);
                        m1.x = fmaxf(m1.x, v1.x); m1.y = fmaxf(m1.y, v1.y); m1.z = fmaxf(m1.z, v1.z); m1.w = fmaxf(m1.w, v1.w);
                    }
                const int py = PT3 * ty + pi, px = PT3 * tx + pj;
                const bool ok = item && py < a.ph && px < a.pw;
                const unsigned off = ok ? (unsigned)(((py * a.pw + px) * 64 + 8 * ch) * 4) : 0x80000000u;
                // unconditional (dropped past the map): every thread issues exactly 4 stores per tile
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, m0), ry, off, 0, 0);
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, m1), ry, off + 16u, 0, 0);
                if (ok)
                    tm = fmaxf(tm, fmaxf(fmaxf(fmaxf(m0.x, m0.y), fmaxf(m0.z, m0.w)),
                                         fmaxf(fmaxf(m1.x, m1.y), fmaxf(m1.z, m1.w))));
            }
            if (a.ymax) amax_lds_add(s_amax, b, tm);          // the tile's frame: block-uniform
        }
    }
    if (a.ymax) {
        __syncthreads();
        amax_lds_flush(s_amax, a.ymax, a.B);
    }
}

}  // namespace

hipError_t vd_launch_stem_pool32(const StemPoolArgs& a, hipStream_t s) {
    if (a.B <= 0) return hipSuccess;
    if (a.B > 1024) return hipErrorInvalidValue;
    const size_t lds = 2 * XBUF3 + STB3 + 1024 + 4 * (size_t)a.B;
    static const int cus = [] {
        (void)hipFuncSetAttribute((const void*)stem_pool32_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  2 * XBUF3 + STB3 + 1024 + 4 * 1024);
        int dev = 0, n = 256;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
        return n > 0 ? n : 256;
    }();
    const int tiles = a.B * ((a.ph + PT3 - 1) / PT3) * ((a.pw + PT3 - 1) / PT3);
    const int grid = tiles < 2 * cus ? tiles : 2 * cus;   // persistent, two workgroups per CU
    hipLaunchKernelGGL(stem_pool32_kernel, dim3(grid), dim3(256), lds, s, a);
    return hipGetLastError();
}
