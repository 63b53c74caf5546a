// block32.hip — one whole ResNet-50 layer1 bottleneck in one kernel, fp32 plan.
//
// torchvision Bottleneck [ext] (torchvision/models/resnet.py, v1.5) as built from
// the reference's body.layer1.* weights (detect_face/retinaface.py:53-60,
// IntermediateLayerGetter over resnet50), in the arithmetic of the fp32 plan
// (conv_x6.hip: f32 activations and weights, each product as three fp16 MFMA
// products of power-of-two-scaled hi/lo pairs, f32 accumulation):
//   t1  = relu(bn1(conv1x1(x)))            64 ch, on the 10x18 halo of the tile
//   t2  = relu(bn2(conv3x3(t1, pad 1)))    64 ch
//   out = relu(bn3(conv1x1(t2)) + idt)     256 ch; idt = x (layer1.1, layer1.2) or
//                                          bn(downsample(x)) (layer1.0, CIN = 64)
// Conv-by-conv, each layer1 block moves ~6.7 GB of f32 tensors per 64 frames
// through HBM (x twice, t1 and t2 out and back, out once); here t1 and t2 never
// leave LDS: x is read once (its halo neighbours from L2) and out written once.
//
// Operand scales. x keeps its producer's per-frame scale (Act::amax, as every
// fp32-plan conv). t1 and t2 are produced and consumed inside one tile, so each
// takes a per-TILE power of two from the tile's own maximum (an LDS reduction
// before the split): a row of the conv2 / conv3 GEMM keeps one scale over all of
// its K, so the scale still factors out of every dot product exactly; against the
// per-frame scale of the unfused plan it only moves where the fp16 pair rounds
// (f32-level either way; tests/test_gpu_kernels.py compares both with float64).
//
// One workgroup = 8 waves, persistent over 8x16-pixel output tiles of one frame:
//   stage 1  t1^T = W1 . X^T over the 180 halo pixels: wave w owns halo pixel tile w
//            (all 64 channels) and half of tile 8 + w/2 (32 channels); x fragments
//            from global (zeros past the frame by buffer loads), split in registers,
//            W1 planes from LDS. BN+ReLU, zero outside the frame (conv2's padding),
//            tile max -> scale -> hi/lo planes of t1 in LDS.
//   stage 2  t2^T = W2 . T1win^T: wave (jn = w & 3, hf = w >> 2) computes t2 channels
//            16jn.. over all 128 pixels on input channels 32hf.. (split K: its 9 taps x
//            2 planes of W2 fragments stay in VGPRs); every t1 window is read once and
//            feeds the three output rows it touches; the hf = 1 partial sums go through
//            LDS, the hf = 0 waves finish BN+ReLU, tile max -> scale -> t2 planes.
//   stage 3  out = W3 . t2 (+ Wd . x): wave w owns output channels 32w..32w+31 (W3, Wd
//            fragments stationary, rows permuted so a lane holds 8 consecutive
//            channels), one 16-pixel output row at a time; identity / downsample input
//            from global (L2: the halo was just read), BN, ReLU, two 16-B f32 stores
//            per lane, per-frame max |out| into the output's slots.
// LDS: W1 planes (CIN x 64 x 2 fp16, 16 / 64 KB) + t1 planes (192 x 64 x 2 fp16, 48 KB)
// + t2 planes (128 x 64 x 2 fp16, 32 KB; the stage-2 partials before that) + BN tables.
#include "vd_common.h"

namespace {

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

constexpr int TH = 8, TW = 16;                  // output tile
constexpr int HWD = TW + 2;                     // halo width
constexpr int HROWS = (TH + 2) * HWD;           // 180 halo pixels
constexpr int CO = 256;
constexpr int T1PL = 192 * 128;                 // one t1 plane: 192 rows x 64 fp16
constexpr int T2PL = 128 * 128;                 // one t2 plane

// 128-B rows of 64 fp16 channels, 16-B chunk c of row r at c ^ (2 * ((r >> 1) & 3)):
// conflict-free ds_read_b128 for any 16 consecutive rows (block.hip)
__device__ __forceinline__ int lds_off(int row, int chunk) {
    return row * 128 + ((chunk ^ (((row >> 1) & 3) << 1)) << 4);
}
// 64-B rows (32 fp16 of one k-step) of the W1 image: conv_x6.hip's swizzle
__device__ __forceinline__ int swz64(int row, int chunk) { return row * 64 + ((chunk ^ (((row >> 3) & 1) * 3)) << 4); }

__device__ __forceinline__ f32x4_t mfma_pair(const u32x4 (&a)[2], const u32x4 (&b)[2], f32x4_t acc) {
    // (a_hi + a_lo)(b_hi + b_lo) without a_lo b_lo, small terms first
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8_t, a[1]), __builtin_bit_cast(f16x8_t, b[0]),
                                                 acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8_t, a[0]), __builtin_bit_cast(f16x8_t, b[1]),
                                                 acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8_t, a[0]), __builtin_bit_cast(f16x8_t, b[0]),
                                                 acc, 0, 0, 0);
    return acc;
}

// 8 f32 (already in registers as two u32x4) -> fp16 hi / lo planes of x * sa
__device__ __forceinline__ void split8(const u32x4& a, const u32x4& b, float sa, u32x4 (&o)[2]) {
    unsigned h[8], l[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const float x = __uint_as_float(j < 4 ? a[j] : b[j - 4]);
        const _Float16 x0 = (_Float16)__builtin_fmaf(x, sa, 0.f);
        const _Float16 x1 = (_Float16)__builtin_fmaf(x, sa, -(float)x0);
        h[j] = __builtin_bit_cast(unsigned short, x0);
        l[j] = __builtin_bit_cast(unsigned short, x1);
    }
    o[0] = u32x4{h[0] | (h[1] << 16), h[2] | (h[3] << 16), h[4] | (h[5] << 16), h[6] | (h[7] << 16)};
    o[1] = u32x4{l[0] | (l[1] << 16), l[2] | (l[3] << 16), l[4] | (l[5] << 16), l[6] | (l[7] << 16)};
}

// 4 f32 -> 4 fp16 hi and 4 fp16 lo (8 B each)
__device__ __forceinline__ void split4(const float (&v)[4], float sa, u32x2& hi, u32x2& lo) {
    unsigned h[4], l[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const _Float16 x0 = (_Float16)__builtin_fmaf(v[j], sa, 0.f);
        const _Float16 x1 = (_Float16)__builtin_fmaf(v[j], sa, -(float)x0);
        h[j] = __builtin_bit_cast(unsigned short, x0);
        l[j] = __builtin_bit_cast(unsigned short, x1);
    }
    hi = u32x2{h[0] | (h[1] << 16), h[2] | (h[3] << 16)};
    lo = u32x2{l[0] | (l[1] << 16), l[2] | (l[3] << 16)};
}

// power-of-two exponent k with m * 2^k in [2^14, 2^15) (act_scale_exp's rule)
__device__ __forceinline__ int scale_exp(float m) {
    if (!(m > 0.f) || !(m < 3.0e38f)) return 0;
    int e;
    (void)frexpf(m, &e);
    const int k = 15 - e;
    return k < -100 ? -100 : (k > 100 ? 100 : k);
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
    return v;
}

template <int CIN, bool DS, int XD>
__global__ __launch_bounds__(512, 1) void bottleneck32_kernel(Block32Args a) {
    constexpr int KS1 = CIN / 32;                         // stage-1 k-steps
    // stage-1 x register sets: k-step s + XD - 1 is issued while s is split and
    // multiplied (the loads are HBM latency bound: one k-step of MFMA work is a small
    // fraction of a load's round trip)
    static_assert(XD >= 2 && XD <= KS1, "stage-1 x depth");
    constexpr int W1PL = KS1 * 64 * 64;                   // one W1 plane
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* lw1 = smem;
    char* lt1 = lw1 + 2 * W1PL;
    char* lt2 = lt1 + 2 * T1PL;
    float* s_bn = (float*)(lt2 + 2 * T2PL);               // s1 h1 s2 h2 (64 each), s3 h3 (sd hd) (256 each)
    unsigned* s_max = (unsigned*)(s_bn + 256 + 512 * (DS ? 2 : 1));   // [0] t1 max, [1] t2 max

    const int tid = threadIdx.x, lane = tid & 63, li0 = lane & 15, g0 = lane >> 4;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int jn = w & 3, hf = w >> 2;
    const int tpf = a.tiles_x * a.tiles_y, T = a.B * tpf;
    // each XCD takes a contiguous tile range (halo neighbours share its L2)
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
    if (t0 >= tend) return;

    // ---- workgroup constants: W1 planes and BN tables into LDS ----
    for (int i = tid; i < 2 * KS1 * 64 * 4; i += 512) {   // 16-B pieces: [plane][ks][row][chunk]
        const int c = i & 3, row = (i >> 2) & 63, pk = i >> 8, ks = pk % KS1, p = pk / KS1;
        const u32x4 v = *(const u32x4*)((const char*)a.w1 + ((size_t)(p * KS1 + ks) * 64 + row) * 64 + c * 16);
        *(u32x4*)(lw1 + p * W1PL + ks * 4096 + swz64(row, c)) = v;
    }
    for (int i = tid; i < 256 + 512 * (DS ? 2 : 1); i += 512) s_bn[i] = a.bn[i];
    if (tid < 2) s_max[tid] = 0u;
    const float* s1 = s_bn;
    const float* h1 = s_bn + 64;
    const float* s2 = s_bn + 128;
    const float* h2 = s_bn + 192;
    const float* s3 = s_bn + 256;
    const float* h3 = s_bn + 512;
    const float* sd = s_bn + 768;
    const float* hd = s_bn + 1024;

    // stationary fragments: W2 (this wave's 16 channels x its input half, 9 taps x 2
    // planes). W3 / Wd (its 32 output channels, 2 tiles x 2 k-steps x 2 planes) are
    // re-read from L2 per tile, issued before the t2 split so they land under it:
    // stationary they would not fit beside W2 and the stage-2 accumulators
    const __amdgpu_buffer_rsrc_t rw2 = __builtin_amdgcn_make_buffer_rsrc((void*)a.w2, 0, 0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t rw3 = __builtin_amdgcn_make_buffer_rsrc((void*)a.w3, 0, 0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t rwd = __builtin_amdgcn_make_buffer_rsrc((void*)(DS ? a.wd : a.w3), 0, 0x7fffffff,
                                                                          0x00020000);
    const unsigned lo16 = (unsigned)lane * 16u;
    u32x4 w2f[9][2];
#pragma unroll
    for (int tp = 0; tp < 9; ++tp)
#pragma unroll
        for (int p = 0; p < 2; ++p)
            w2f[tp][p] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                rw2, lo16, ((((jn * 2 + hf) * 9 + tp) * 2 + p) * 64) * 16, 0));
    const size_t fpx = (size_t)a.H * a.W;
    int ob = -1;            // output max bookkeeping: this wave's current frame and its max
    float om = 0.f;

    // stage-1 x of halo pixel tiles w and 8 + w/2 (lane: pixel 16 p + li, channels 8 g..)
    auto xoff = [&](int oy0, int ox0, int p, int li, int g) {
        const int r = 16 * p + li;
        const int hy = r / HWD, hx = r - hy * HWD;
        const int iy = oy0 - 1 + hy, ix = ox0 - 1 + hx;
        const bool in = r < HROWS && (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W;
        return in ? (unsigned)((iy * a.W + ix) * CIN + 8 * g) * 4u : 0x80000000u;
    };
    auto ldx = [&](__amdgpu_buffer_rsrc_t rx, unsigned offA, unsigned offB, int s, u32x4 (&ra)[2], u32x4 (&rb)[2]) {
        const int so = s * 128;
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            ra[q] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rx, offA, so + 16 * q, 0));
            rb[q] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rx, offB, so + 16 * q, 0));
        }
    };
    auto frame_rsrc = [&](int b) {
        return __builtin_amdgcn_make_buffer_rsrc((void*)((const float*)a.x + (size_t)b * fpx * CIN), 0,
                                                 (int)(fpx * CIN * 4), 0x00020000);
    };

#pragma unroll 1
    for (int t = t0; t < tend; t += tstep) {
        const int b = t / tpf, r0 = t - b * tpf;
        const int ty = r0 / a.tiles_x, tx = r0 - ty * a.tiles_x;
        const int oy0 = ty * TH, ox0 = tx * TW;
        const int kx = scale_exp(__uint_as_float(a.xmax[b]));
        const float sax = __builtin_ldexpf(1.f, kx), invx = __builtin_ldexpf(1.f, -kx);
        const __amdgpu_buffer_rsrc_t rx = frame_rsrc(b);
        __syncthreads();   // B0: the previous tile is done with t1 / t2 / the max slots
        // lane coordinates made opaque per tile: keeps the per-lane LDS / global
        // addresses of the three stages from being hoisted out of the tile loop
        int li = li0, g = g0;
        asm volatile("" : "+v"(li), "+v"(g));

        // ---- stage 1: t1 on halo pixel tiles pA = w (4 channel tiles), pB = 8 + w/2 (2) ----
        float vA[4][4], vB[2][4];
        {
            const int pB = 8 + (w >> 1), hB = w & 1;
            const unsigned offA = xoff(oy0, ox0, w, li, g), offB = xoff(oy0, ox0, pB, li, g);
            f32x4_t accA[4], accB[2];
#pragma unroll
            for (int c = 0; c < 4; ++c) accA[c] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int c = 0; c < 2; ++c) accB[c] = f32x4_t{0.f, 0.f, 0.f, 0.f};
            u32x4 xa[XD][2], xb[XD][2];                  // [set][half]: k-step s in set s % XD
            const int dbg = a.dbg;                       // timing-only stage skips (option block32_dbg)
            if (!(dbg & 1)) {
#pragma unroll
            for (int s = 0; s + 1 < XD; ++s) ldx(rx, offA, offB, s, xa[s], xb[s]);
#pragma unroll
            for (int s = 0; s < KS1; ++s) {
                if (s + XD - 1 < KS1) ldx(rx, offA, offB, s + XD - 1, xa[(s + XD - 1) % XD], xb[(s + XD - 1) % XD]);
                u32x4 pa[2], pb[2];
                split8(xa[s % XD][0], xa[s % XD][1], sax, pa);
                split8(xb[s % XD][0], xb[s % XD][1], sax, pb);
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    u32x4 wf[2];
#pragma unroll
                    for (int p = 0; p < 2; ++p) wf[p] = *(const u32x4*)(lw1 + p * W1PL + s * 4096 + swz64(16 * c + li, g));
                    accA[c] = mfma_pair(wf, pa, accA[c]);
                    if ((c >> 1) == hB) accB[c & 1] = mfma_pair(wf, pb, accB[c & 1]);
                }
            }
            }
            // BN + ReLU, zero outside the frame (conv2's padding) and past the halo
            float m = 0.f;
            auto finish = [&](const f32x4_t& acc, int c, int p, float (&v)[4]) {
                const int r = 16 * p + li;
                const int hy = r / HWD, hx = r - hy * HWD;
                const int iy = oy0 - 1 + hy, ix = ox0 - 1 + hx;
                const bool in = r < HROWS && (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W;
                const float4 sc = *(const float4*)(s1 + 16 * c + 4 * g), sh = *(const float4*)(h1 + 16 * c + 4 * g);
                const float scv[4] = {sc.x, sc.y, sc.z, sc.w}, shv[4] = {sh.x, sh.y, sh.z, sh.w};
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float y = (acc[e] * invx) * scv[e] + shv[e];
                    v[e] = (in && y > 0.f) ? y : 0.f;
                    m = fmaxf(m, v[e]);
                }
            };
#pragma unroll
            for (int c = 0; c < 4; ++c) finish(accA[c], c, w, vA[c]);
#pragma unroll
            for (int c = 0; c < 2; ++c) finish(accB[c], 2 * hB + c, pB, vB[c]);
            m = wave_max(m);
            if (lane == 0 && m > 0.f) atomicMax(s_max, __float_as_uint(m));
        }
        __syncthreads();   // B1: the tile's t1 max is complete
        {
            const int pB = 8 + (w >> 1), hB = w & 1;
            const float sa1 = __builtin_ldexpf(1.f, scale_exp(__uint_as_float(s_max[0])));
            auto store = [&](const float (&v)[4], int c, int p) {
                u32x2 hi, lo;
                split4(v, sa1, hi, lo);
                const int off = lds_off(16 * p + li, 2 * c + (g >> 1)) + (g & 1) * 8;
                *(u32x2*)(lt1 + off) = hi;
                *(u32x2*)(lt1 + T1PL + off) = lo;
            };
#pragma unroll
            for (int c = 0; c < 4; ++c) store(vA[c], c, w);
#pragma unroll
            for (int c = 0; c < 2; ++c) store(vB[c], 2 * hB + c, pB);
            if (tid == 0) s_max[1] = 0u;             // t2's max: last read before this tile's B0
        }
        const int k1 = scale_exp(__uint_as_float(s_max[0]));
        __syncthreads();   // B2: t1 planes complete
        if (tid == 0) s_max[0] = 0u;                 // read by every wave before B2

        // ---- stage 2: t2^T channels 16jn.. over the 8 output rows, input half hf ----
        f32x4_t acc2[8];
#pragma unroll
        for (int m = 0; m < 8; ++m) acc2[m] = f32x4_t{0.f, 0.f, 0.f, 0.f};
        {
            // window q = (halo row hh = q / 3, shift dx = q % 3), both planes; read once,
            // used by output rows m = hh - dy; reads run PD windows ahead
            constexpr int PD = 2;
            u32x4 tf[PD + 1][2];
#define VD_T1READ(Q)                                                                                   \
            do {                                                                                       \
                const int hh_ = (Q) / 3, dx_ = (Q) % 3;                                                \
                const int off_ = lds_off(hh_ * HWD + li + dx_, 4 * hf + g);                            \
                tf[(Q) % (PD + 1)][0] = *(const u32x4*)(lt1 + off_);                                   \
                tf[(Q) % (PD + 1)][1] = *(const u32x4*)(lt1 + T1PL + off_);                            \
            } while (0)
            if (!(a.dbg & 2)) {
#pragma unroll
            for (int q = 0; q < PD; ++q) VD_T1READ(q);
#pragma unroll
            for (int q = 0; q < 30; ++q) {
                asm volatile("" ::: "memory");
                if (q + PD < 30) VD_T1READ(q + PD);
                const int hh = q / 3, dx = q % 3;
#pragma unroll
                for (int dy = 0; dy < 3; ++dy) {
                    const int m = hh - dy;
                    if (m >= 0 && m < 8) acc2[m] = mfma_pair(w2f[3 * dy + dx], tf[q % (PD + 1)], acc2[m]);
                }
            }
            }
#undef VD_T1READ
        }
        // split-K: the hf = 1 partial sums -> LDS (the t2 region, free until B4)
        float* part = (float*)lt2;
        if (hf == 1) {
#pragma unroll
            for (int m = 0; m < 8; ++m) *(f32x4_t*)(part + ((jn * 8 + m) * 64 + lane) * 4) = acc2[m];
        }
        __syncthreads();   // B3: partials in LDS
        // t2 values wait for the tile max in the (now dead) t1 region, not in registers
        f32x4_t* v2s = (f32x4_t*)lt1 + (jn * 8) * 64 + lane;
        const float inv1 = __builtin_ldexpf(1.f, -k1);
        if (hf == 0) {
            const float4 sc = *(const float4*)(s2 + 16 * jn + 4 * g), sh = *(const float4*)(h2 + 16 * jn + 4 * g);
            const float scv[4] = {sc.x, sc.y, sc.z, sc.w}, shv[4] = {sh.x, sh.y, sh.z, sh.w};
            float m2 = 0.f;
#pragma unroll
            for (int m = 0; m < 8; ++m) {
                const f32x4_t o = *(const f32x4_t*)(part + ((jn * 8 + m) * 64 + lane) * 4);
                f32x4_t v;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float y = ((acc2[m][e] + o[e]) * inv1) * scv[e] + shv[e];
                    v[e] = y > 0.f ? y : 0.f;
                    m2 = fmaxf(m2, v[e]);
                }
                v2s[m * 64] = v;
            }
            m2 = wave_max(m2);
            if (lane == 0 && m2 > 0.f) atomicMax(s_max + 1, __float_as_uint(m2));
        }
        __syncthreads();   // B4: partials consumed, t2 max complete
        const int k2 = scale_exp(__uint_as_float(s_max[1]));
        if (hf == 0) {
            const float sa2 = __builtin_ldexpf(1.f, k2);
#pragma unroll
            for (int m = 0; m < 8; ++m) {
                u32x2 hi, lo;
                const f32x4_t v = v2s[m * 64];
                const float vv[4] = {v[0], v[1], v[2], v[3]};
                split4(vv, sa2, hi, lo);
                const int off = lds_off(16 * m + li, 2 * jn + (g >> 1)) + (g & 1) * 8;
                *(u32x2*)(lt2 + off) = hi;
                *(u32x2*)(lt2 + T2PL + off) = lo;
            }
        }
        // this tile's W3 / Wd fragments, issued after the t2 split (its values are dead
        // by then) so they land under B5 (the lane offset made opaque per tile, so the
        // loads are not hoisted out of the tile loop into 64 live registers)
        u32x4 w3f[2][2][2], wdf[DS ? 2 : 1][DS ? 2 : 1][2];
        {
            unsigned lo = lo16;
            asm volatile("" : "+v"(lo));
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int s = 0; s < 2; ++s)
#pragma unroll
                    for (int p = 0; p < 2; ++p) {
                        const int so = ((((w * 2 + j) * 2 + s) * 2 + p) * 64) * 16;
                        w3f[j][s][p] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rw3, lo, so, 0));
                        if constexpr (DS)
                            wdf[j][s][p] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rwd, lo, so, 0));
                    }
        }
        // ---- stage 3 operands in flight across B5: the first identity row (below) ----
        const int c0 = 32 * w + 8 * g;
        const int ox = ox0 + li;
        // per output row: identity x[px][c0..c0+7] (2 x 16 B), or the downsample
        // input x[px][32 s + 8 g ..] (2 k-steps x 2 x 16 B); prefetched one row ahead
        constexpr int NX = DS ? 4 : 2;
        u32x4 xr[DS ? 1 : 2][NX];        // DS: no prefetch (registers)
        auto ldr = [&](int m, u32x4 (&r)[NX]) {
            const int oy = oy0 + m;
            const bool in = oy < a.H && ox < a.W;
            if constexpr (DS) {
                const unsigned o = in ? (unsigned)((oy * a.W + ox) * CIN + 8 * g) * 4u : 0x80000000u;
#pragma unroll
                for (int s = 0; s < 2; ++s)
#pragma unroll
                    for (int q = 0; q < 2; ++q)
                        r[2 * s + q] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                            rx, o, s * 128 + 16 * q, 0));
            } else {
                const unsigned o = in ? (unsigned)((oy * a.W + ox) * CIN + c0) * 4u : 0x80000000u;
#pragma unroll
                for (int q = 0; q < 2; ++q)
                    r[q] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rx, o, 16 * q, 0));
            }
        };
        if constexpr (!DS) ldr(0, xr[0]);
        __syncthreads();   // B5: t2 planes complete

        // ---- stage 3: out channels 32w + 8g .. +7 per lane, 8 output rows ----
        {
            const float inv2 = __builtin_ldexpf(1.f, -k2);
            const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc(
                (void*)((float*)a.y + (size_t)b * fpx * CO), 0, (int)(fpx * CO * 4), 0x00020000);
            float om_t = 0.f;
#pragma unroll
            for (int m = 0; m < 8; ++m) {
                __builtin_amdgcn_sched_barrier(0);   // keep rows apart (register pressure)
                if (!(a.dbg & 16)) { if constexpr (DS) ldr(m, xr[0]); else if (m + 1 < 8) ldr(m + 1, xr[(m + 1) & 1]); }
                f32x4_t acc[2] = {f32x4_t{0.f, 0.f, 0.f, 0.f}, f32x4_t{0.f, 0.f, 0.f, 0.f}};
                if (!(a.dbg & 4)) {
                u32x4 tfr[2][2];
#pragma unroll
                for (int s = 0; s < 2; ++s) {
                    const int off = lds_off(16 * m + li, 4 * s + g);
                    tfr[s][0] = *(const u32x4*)(lt2 + off);
                    tfr[s][1] = *(const u32x4*)(lt2 + T2PL + off);
                }
#pragma unroll
                for (int j = 0; j < 2; ++j)
#pragma unroll
                    for (int s = 0; s < 2; ++s) acc[j] = mfma_pair(w3f[j][s], tfr[s], acc[j]);
                }
                float v[8];
                int cb = c0;                          // BN tables re-read per row (LDS), not held
                asm volatile("" : "+v"(cb));
                {
                    const float4 sa = *(const float4*)(s3 + cb), sb = *(const float4*)(s3 + cb + 4);
                    const float4 ha = *(const float4*)(h3 + cb), hb = *(const float4*)(h3 + cb + 4);
                    const float scv[8] = {sa.x, sa.y, sa.z, sa.w, sb.x, sb.y, sb.z, sb.w};
                    const float shv[8] = {ha.x, ha.y, ha.z, ha.w, hb.x, hb.y, hb.z, hb.w};
#pragma unroll
                    for (int e = 0; e < 8; ++e) v[e] = (acc[e >> 2][e & 3] * inv2) * scv[e] + shv[e];
                }
                const u32x4* xc = xr[DS ? 0 : (m & 1)];
                if constexpr (DS) {   // + bn_d(downsample(x)), rounded to f32 first (the unfused plan's stored value)
                    f32x4_t accd[2] = {f32x4_t{0.f, 0.f, 0.f, 0.f}, f32x4_t{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
                    for (int s = 0; s < 2; ++s) {
                        u32x4 px[2];
                        split8(xc[2 * s], xc[2 * s + 1], sax, px);
#pragma unroll
                        for (int j = 0; j < 2; ++j) accd[j] = mfma_pair(wdf[j][s], px, accd[j]);
                    }
                    const float4 sa = *(const float4*)(sd + cb), sb = *(const float4*)(sd + cb + 4);
                    const float4 ha = *(const float4*)(hd + cb), hb = *(const float4*)(hd + cb + 4);
                    const float scv[8] = {sa.x, sa.y, sa.z, sa.w, sb.x, sb.y, sb.z, sb.w};
                    const float shv[8] = {ha.x, ha.y, ha.z, ha.w, hb.x, hb.y, hb.z, hb.w};
#pragma unroll
                    for (int e = 0; e < 8; ++e) v[e] += (accd[e >> 2][e & 3] * invx) * scv[e] + shv[e];
                } else {              // + identity
#pragma unroll
                    for (int e = 0; e < 8; ++e) v[e] += __uint_as_float(xc[e >> 2][e & 3]);
                }
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    v[e] = v[e] > 0.f ? v[e] : 0.f;
                    om_t = fmaxf(om_t, v[e]);
                }
                const int oy = oy0 + m;
                const unsigned so = (oy < a.H && ox < a.W && !(a.dbg & 8)) ? (unsigned)((oy * a.W + ox) * CO + c0) * 4u
                                                                           : 0x80000000u;
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, f32x4_t{v[0], v[1], v[2], v[3]}), ry,
                                                       so, 0, 0);
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, f32x4_t{v[4], v[5], v[6], v[7]}), ry,
                                                       so, 16, 0);
            }
            // per-frame max |out| (values are >= 0): one atomic per wave per frame change
            om_t = wave_max(om_t);
            if (b != ob) {
                if (ob >= 0 && lane == 0 && om > 0.f) atomicMax(a.ymax + ob, __float_as_uint(om));
                ob = b;
                om = 0.f;
            }
            om = fmaxf(om, om_t);
        }
    }
    if (ob >= 0 && lane == 0 && om > 0.f) atomicMax(a.ymax + ob, __float_as_uint(om));
}

// ---------------------------------------------------------------------------------
// Pipelined form (option block32_pipe, default 1; layer1.1 / layer1.2, CIN = 256): the
// same three stages, tiles, products and operand scales, on twelve waves in three groups
// of four that work on CONSECUTIVE tiles at once, so neither the x stream from HBM nor
// the output stores stop at a workgroup barrier:
//   P (waves 0-3):  stage 1 of tile j+1 -- wave w: halo pixel tiles 3w..3w+2, all 64 t1
//                   channels, W1 planes from LDS, x two k-steps deep and the next tile's
//                   first k-step issued before the t1 hand-over;
//   C (waves 4-7):  stage 2 of tile j -- the wave owns t2 channels 16jn.. over the full
//                   K = 9 taps x 64; its W2 taps re-read from L2 as the previous K half's
//                   taps fall dead;
//   Q (waves 8-11): stage 3 of tile j-1 -- the wave owns output channels 64jn.., two
//                   32-channel groups one after the other, W3 per group from L2 and the
//                   group's eight identity rows issued before its stores (CDNA4's vmcnt
//                   retires loads and stores in issue order: a load issued behind a store
//                   waits for it).
// t1 and t2 cross between the groups through single LDS plane buffers, split once by
// their producer (each holds its values in registers until the buffer is free); the
// per-tile max is a counter barrier among the four producing waves. Six monotonic LDS
// counters (t1 ready / free, t2 ready / free, P max, C max; waits spin with s_sleep)
// replace the workgroup barriers. Stage 2 sums each output's 18 k-steps in one
// accumulator instead of two K halves (f32 rounding; tests/test_gpu_e2e.py,
// test_gpu_kernels.py).

__device__ __forceinline__ int lds_load_flag(int* f) {
    return __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// wait until *f >= v (the LDS data behind the counter was written before it was bumped)
__device__ __forceinline__ void wait_flag(int* f, int v) {
    while (__builtin_amdgcn_readfirstlane(lds_load_flag(f)) < v) __builtin_amdgcn_s_sleep(1);
    asm volatile("" ::: "memory");
}
// this wave's LDS writes / reads are complete, then bump the counter (one lane)
__device__ __forceinline__ void post_flag(int* f, int lane) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (lane == 0) __hip_atomic_fetch_add(f, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    asm volatile("" ::: "memory");
}

template <int CIN, int XS, int PRE>
__global__ __launch_bounds__(768, 1) void bottleneck32p_kernel(Block32Args a) {
    constexpr int KS1 = CIN / 32;
    constexpr int W1PL = KS1 * 64 * 64;                   // one W1 plane
    constexpr int NP = 3;                                 // halo pixel tiles per producer wave
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* lw1 = smem;                                     // W1 planes (as the one-group kernel)
    char* lt1 = lw1 + 2 * W1PL;                           // t1 hi / lo planes (as the one-group kernel)
    char* lt2 = lt1 + 2 * T1PL;                           // t2 hi / lo planes
    float* s_bn = (float*)(lt2 + 2 * T2PL);               // s1 h1 s2 h2 (64 each), s3 h3 (256 each)
    int* s_flag = (int*)(s_bn + 768);                     // t1 ready, t1 free, t2 ready, t2 free, P max, C max
    unsigned* s_t1max = (unsigned*)(s_flag + 8);          // [4] per-tile max |t1| (slot = tile & 3)
    unsigned* s_t2max = s_t1max + 4;                      // [4]

    const int tid = threadIdx.x, lane = tid & 63, li0 = lane & 15, g0 = lane >> 4;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int tpf = a.tiles_x * a.tiles_y, T = a.B * tpf;
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
    if (t0 >= tend) return;
    const int ntile = (tend - t0 + tstep - 1) / tstep;
    for (int i = tid; i < 2 * KS1 * 64 * 4; i += 768) {   // 16-B pieces: [plane][ks][row][chunk]
        const int c = i & 3, row = (i >> 2) & 63, pk = i >> 8, ks = pk % KS1, p = pk / KS1;
        const u32x4 v = *(const u32x4*)((const char*)a.w1 + ((size_t)(p * KS1 + ks) * 64 + row) * 64 + c * 16);
        *(u32x4*)(lw1 + p * W1PL + ks * 4096 + swz64(row, c)) = v;
    }
    for (int i = tid; i < 768; i += 768) s_bn[i] = a.bn[i];
    if (tid < 16) s_flag[tid] = 0;                        // counters and both max slot rings
    __syncthreads();
    const float* s1 = s_bn;
    const float* h1 = s_bn + 64;
    const float* s2 = s_bn + 128;
    const float* h2 = s_bn + 192;
    const float* s3 = s_bn + 256;
    const float* h3 = s_bn + 512;
    const size_t fpx = (size_t)a.H * a.W;
    const unsigned lo16 = (unsigned)lane * 16u;
    auto frame_rsrc = [&](int b) {
        return __builtin_amdgcn_make_buffer_rsrc((void*)((const float*)a.x + (size_t)b * fpx * CIN), 0,
                                                 (int)(fpx * CIN * 4), 0x00020000);
    };
    auto tile_of = [&](int j, int& b, int& oy0, int& ox0) {
        const int t = t0 + j * tstep;
        b = t / tpf;
        const int r0 = t - b * tpf, ty = r0 / a.tiles_x;
        oy0 = ty * TH;
        ox0 = (r0 - ty * a.tiles_x) * TW;
    };

    if (w < 4) {
        // ================= producer: stage 1 of tile j =================
        // x of halo pixel tile 3w + i (lane: pixel 16 (3w + i) + li, channels 8g..), k-step s
        auto xoff = [&](int oy0, int ox0, int i, int li, int g) {
            const int r = 16 * (NP * w + i) + li;
            const int hy = r / HWD, hx = r - hy * HWD;
            const int iy = oy0 - 1 + hy, ix = ox0 - 1 + hx;
            const bool in = r < HROWS && (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W;
            return in ? (unsigned)((iy * a.W + ix) * CIN + 8 * g) * 4u : 0x80000000u;
        };
        auto ldx = [&](__amdgpu_buffer_rsrc_t rx, const unsigned (&off)[NP], int s, u32x4 (&r)[NP][2]) {
#pragma unroll
            for (int i = 0; i < NP; ++i)
#pragma unroll
                for (int q = 0; q < 2; ++q)
                    r[i][q] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rx, off[i], s * 128 + 16 * q, 0));
        };
        // k-steps 0 .. PRE-1 of the next stage 1, issued before the current tile's t1 hand-over
        // XS x register sets: XS - 1 k-steps in flight; PRE of them issued before the hand-over
        static_assert(PRE >= 1 && PRE < XS && XS <= KS1, "stage-1 x depth");
        u32x4 xpre[PRE][NP][2];
        {
            int b, oy0, ox0;
            tile_of(0, b, oy0, ox0);
            unsigned off[NP];
#pragma unroll
            for (int i = 0; i < NP; ++i) off[i] = xoff(oy0, ox0, i, li0, g0);
#pragma unroll
            for (int s = 0; s < PRE; ++s) ldx(frame_rsrc(b), off, s, xpre[s]);
        }
#pragma unroll 1
        for (int j = 0; j < ntile; ++j) {
            {
                // ---- stage 1: t1 of halo pixel tiles 3w..3w+2, all 64 channels ----
                int b, oy0, ox0;
                tile_of(j, b, oy0, ox0);
                const int kx = scale_exp(__uint_as_float(a.xmax[b]));
                const float sax = __builtin_ldexpf(1.f, kx), invx = __builtin_ldexpf(1.f, -kx);
                const __amdgpu_buffer_rsrc_t rx = frame_rsrc(b);
                int li = li0, g = g0;
                asm volatile("" : "+v"(li), "+v"(g));
                unsigned off[NP];
#pragma unroll
                for (int i = 0; i < NP; ++i) off[i] = xoff(oy0, ox0, i, li, g);
                f32x4_t acc[NP][4];
#pragma unroll
                for (int i = 0; i < NP; ++i)
#pragma unroll
                    for (int c = 0; c < 4; ++c) acc[i][c] = f32x4_t{0.f, 0.f, 0.f, 0.f};
                u32x4 xs[XS][NP][2];                       // k-step s in set s % XS
#pragma unroll
                for (int s = 0; s < PRE; ++s)
#pragma unroll
                    for (int i = 0; i < NP; ++i)
#pragma unroll
                        for (int q = 0; q < 2; ++q) xs[s][i][q] = xpre[s][i][q];
#pragma unroll
                for (int s = PRE; s + 1 < XS; ++s) ldx(rx, off, s, xs[s]);
                if (!(a.dbg & 1))                          // timing-only skip (option block32_dbg)
#pragma unroll
                for (int ks = 0; ks < KS1; ++ks) {
                    if (ks + XS - 1 < KS1) ldx(rx, off, ks + XS - 1, xs[(ks + XS - 1) % XS]);
                    u32x4 px[NP][2];
#pragma unroll
                    for (int i = 0; i < NP; ++i) split8(xs[ks % XS][i][0], xs[ks % XS][i][1], sax, px[i]);
#pragma unroll
                    for (int c = 0; c < 4; ++c) {
                        u32x4 wf[2];
#pragma unroll
                        for (int p = 0; p < 2; ++p) wf[p] = *(const u32x4*)(lw1 + p * W1PL + ks * 4096 + swz64(16 * c + li, g));
#pragma unroll
                        for (int i = 0; i < NP; ++i) acc[i][c] = mfma_pair(wf, px[i], acc[i][c]);
                    }
                }
                // BN + ReLU, zero outside the frame (conv2's padding); values stay in acc
                const float4* s1v = (const float4*)s1;
                float m = 0.f;
#pragma unroll
                for (int i = 0; i < NP; ++i) {
                    const int r = 16 * (NP * w + i) + li;
                    const int hy = r / HWD, hx = r - hy * HWD;
                    const int iy = oy0 - 1 + hy, ix = ox0 - 1 + hx;
                    const bool in = r < HROWS && (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W;
#pragma unroll
                    for (int c = 0; c < 4; ++c) {
                        const float4 sc = s1v[4 * c + g], sh = *(const float4*)(h1 + 16 * c + 4 * g);
                        const float scv[4] = {sc.x, sc.y, sc.z, sc.w}, shv[4] = {sh.x, sh.y, sh.z, sh.w};
#pragma unroll
                        for (int e = 0; e < 4; ++e) {
                            const float y = (acc[i][c][e] * invx) * scv[e] + shv[e];
                            acc[i][c][e] = (in && y > 0.f) ? y : 0.f;
                            m = fmaxf(m, acc[i][c][e]);
                        }
                    }
                }
                // the next tile's first k-step, in flight across the t1 hand-over
                if (j + 1 < ntile) {
                    int b2, oy2, ox2;
                    tile_of(j + 1, b2, oy2, ox2);
                    unsigned off2[NP];
#pragma unroll
                    for (int i = 0; i < NP; ++i) off2[i] = xoff(oy2, ox2, i, li, g);
#pragma unroll
                    for (int s = 0; s < PRE; ++s) ldx(frame_rsrc(b2), off2, s, xpre[s]);
                }
                // the tile's t1 max over the four producers (counter barrier), its scale, and the
                // split into the hi / lo planes once, here (the consumers read pairs directly)
                m = wave_max(m);
                if (lane == 0 && m > 0.f) atomicMax(s_t1max + (j & 3), __float_as_uint(m));
                post_flag(s_flag + 4, lane);
                wait_flag(s_flag + 4, 4 * (j + 1));
                const float sa1 = __builtin_ldexpf(1.f, scale_exp(__uint_as_float(s_t1max[j & 3])));
                if (j >= 1) wait_flag(s_flag + 1, 4 * j);  // consumers are done with the t1 planes
#pragma unroll
                for (int i = 0; i < NP; ++i)
#pragma unroll
                    for (int c = 0; c < 4; ++c) {
                        const float v[4] = {acc[i][c][0], acc[i][c][1], acc[i][c][2], acc[i][c][3]};
                        u32x2 hi, lo;
                        split4(v, sa1, hi, lo);
                        const int off = lds_off(16 * (NP * w + i) + li, 2 * c + (g >> 1)) + (g & 1) * 8;
                        *(u32x2*)(lt1 + off) = hi;
                        *(u32x2*)(lt1 + T1PL + off) = lo;
                    }
                post_flag(s_flag + 0, lane);               // t1 ready
            }
        }
    } else if (w < 8) {
        // ================= C: stage 2 of tile j =================
        const int jn = w - 4;
        const __amdgpu_buffer_rsrc_t rw2 = __builtin_amdgcn_make_buffer_rsrc((void*)a.w2, 0, 0x7fffffff, 0x00020000);
        // W2 fragments of K half hf (9 taps x 2 planes), re-read per tile from L2 (all of W2
        // stationary is 144 VGPRs: past the 168 of three waves per SIMD)
        // (taps tp0 .. tp0 + nt - 1 of half hf into f)
        auto ldw2 = [&](int hf, int tp0, int nt, u32x4 (&f)[9][2]) {
            unsigned lo = lo16;
            asm volatile("" : "+v"(lo));
#pragma unroll
            for (int tp = tp0; tp < tp0 + nt; ++tp)
#pragma unroll
                for (int p = 0; p < 2; ++p)
                    f[tp][p] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                        rw2, lo, ((((jn * 2 + hf) * 9 + tp) * 2 + p) * 64) * 16, 0));
        };
#pragma unroll 1
        for (int j = 0; j < ntile; ++j) {
            int b, oy0, ox0;
            tile_of(j, b, oy0, ox0);
            u32x4 w2f[9][2];
            ldw2(0, 0, 9, w2f);
            wait_flag(s_flag + 0, 4 * (j + 1));            // t1 of tile j written
            const int k1 = scale_exp(__uint_as_float(s_t1max[j & 3]));
            if (jn == 0 && lane == 0 && j >= 2) s_t1max[(j - 2) & 3] = 0u;   // read by every consumer already
            const float inv1 = __builtin_ldexpf(1.f, -k1);
            int li = li0, g = g0;
            asm volatile("" : "+v"(li), "+v"(g));
            f32x4_t acc2[8];
#pragma unroll
            for (int m = 0; m < 8; ++m) acc2[m] = f32x4_t{0.f, 0.f, 0.f, 0.f};
            // step i = (K half hf = i / 30, window q = i % 30), one step ahead; a window (halo
            // row hh, shift dx) feeds the output rows m = hh - dy it touches
            u32x4 tr[2][2];                                // [buffer][plane]
            auto rd = [&](int i, u32x4 (&d)[2]) {
                const int hf = i / 30, q = i % 30;
                int l = li;                                // address computed here, not hoisted (registers)
                asm volatile("" : "+v"(l));
                const int off = lds_off((q / 3) * HWD + l + q % 3, 4 * hf + g);
                d[0] = *(const u32x4*)(lt1 + off);
                d[1] = *(const u32x4*)(lt1 + T1PL + off);
            };
            rd(0, tr[0]);
#pragma unroll
            for (int i = 0; i < 60; ++i) {
                asm volatile("" ::: "memory");
                // the second half's taps replace the first half's as they fall dead: taps 3 dy + dx
                // are last used by window row hh = 7 + dy of the first half, first by hh = dy
                if (i == 24) ldw2(1, 0, 3, w2f);
                if (i == 27) ldw2(1, 3, 3, w2f);
                if (i == 30) ldw2(1, 6, 3, w2f);
                if (i + 1 < 60) rd(i + 1, tr[(i + 1) & 1]);
                if (i == 59) post_flag(s_flag + 1, lane);  // the t1 buffer read completely
                const int hf = i / 30, q = i % 30;
                const int hh = q / 3, dx = q % 3;
#pragma unroll
                for (int dy = 0; dy < 3; ++dy) {
                    const int m = hh - dy;
                    if (m >= 0 && m < 8 && !(a.dbg & 2)) acc2[m] = mfma_pair(w2f[3 * dy + dx], tr[i & 1], acc2[m]);
                }
            }
            // BN + ReLU (values stay in acc2 until the t2 buffer is free); tile max into its slot
            {
                const float4 sc = *(const float4*)(s2 + 16 * jn + 4 * g), sh = *(const float4*)(h2 + 16 * jn + 4 * g);
                const float scv[4] = {sc.x, sc.y, sc.z, sc.w}, shv[4] = {sh.x, sh.y, sh.z, sh.w};
                float m2 = 0.f;
#pragma unroll
                for (int m = 0; m < 8; ++m)
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const float y = (acc2[m][e] * inv1) * scv[e] + shv[e];
                        acc2[m][e] = y > 0.f ? y : 0.f;
                        m2 = fmaxf(m2, acc2[m][e]);
                    }
                m2 = wave_max(m2);
                if (lane == 0 && m2 > 0.f) atomicMax(s_t2max + (j & 3), __float_as_uint(m2));
                post_flag(s_flag + 5, lane);               // the tile's t2 max over the four consumers
                wait_flag(s_flag + 5, 4 * (j + 1));
                const float sa2 = __builtin_ldexpf(1.f, scale_exp(__uint_as_float(s_t2max[j & 3])));
                if (j >= 1) wait_flag(s_flag + 3, 4 * j);  // every consumer is done with the t2 planes
#pragma unroll
                for (int m = 0; m < 8; ++m) {
                    const float v[4] = {acc2[m][0], acc2[m][1], acc2[m][2], acc2[m][3]};
                    u32x2 hi, lo;
                    split4(v, sa2, hi, lo);
                    const int off = lds_off(16 * m + li, 2 * jn + (g >> 1)) + (g & 1) * 8;
                    *(u32x2*)(lt2 + off) = hi;
                    *(u32x2*)(lt2 + T2PL + off) = lo;
                }
                post_flag(s_flag + 2, lane);               // this wave's t2 channels written
            }
        }
    } else {
        // ================= Q: stage 3 of tile j =================
        // the wave's 64 output channels as two 32-channel groups, one after the other (t2 read
        // once per group): W3 fragments of the group re-read per tile from L2, the identity of
        // all eight rows issued at the group's start (CDNA4's vmcnt retires loads and stores in
        // issue order: a load issued behind the stores of earlier rows would wait for them)
        const int jn = w - 8;
        const __amdgpu_buffer_rsrc_t rw3 = __builtin_amdgcn_make_buffer_rsrc((void*)a.w3, 0, 0x7fffffff, 0x00020000);
        int ob = -1;
        float om = 0.f;
#pragma unroll 1
        for (int j = 0; j < ntile; ++j) {
            int b, oy0, ox0;
            tile_of(j, b, oy0, ox0);
            int k2 = 0;
            float inv2 = 1.f;
            const __amdgpu_buffer_rsrc_t rx = frame_rsrc(b);
            const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc(
                (void*)((float*)a.y + (size_t)b * fpx * CO), 0, (int)(fpx * CO * 4), 0x00020000);
            int li = li0, g = g0;
            asm volatile("" : "+v"(li), "+v"(g));
            const int ox = ox0 + li;
            float om_t = 0.f;
#pragma unroll 1
            for (int h = 0; h < 2; ++h) {
                u32x4 w3f[2][2][2];                        // [tile][k-step][plane]
                {
                    unsigned lo = lo16;
                    asm volatile("" : "+v"(lo));
#pragma unroll
                    for (int jt = 0; jt < 2; ++jt)
#pragma unroll
                        for (int s = 0; s < 2; ++s)
#pragma unroll
                            for (int p = 0; p < 2; ++p)
                                w3f[jt][s][p] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                    rw3, lo, (((((2 * jn + h) * 2 + jt) * 2 + s) * 2 + p) * 64) * 16, 0));
                }
                const int cb0 = 64 * jn + 32 * h;
                auto ldi = [&](int m, u32x4 (&r)[2]) {     // identity x[px][cb0 + 8g ..]
                    const int oy = oy0 + m;
                    const unsigned o = (oy < a.H && ox < a.W) ? (unsigned)((oy * a.W + ox) * CIN + cb0 + 8 * g) * 4u
                                                               : 0x80000000u;
#pragma unroll
                    for (int q = 0; q < 2; ++q)
                        r[q] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rx, o, 16 * q, 0));
                };
                u32x4 xi[8][2];
#pragma unroll
                for (int m = 0; m < 8; ++m) {
                    if (a.dbg & 16) xi[m][0] = xi[m][1] = u32x4{0u, 0u, 0u, 0u};
                    else ldi(m, xi[m]);
                }
                if (h == 0) {
                    wait_flag(s_flag + 2, 4 * (j + 1));    // t2 of tile j written
                    k2 = scale_exp(__uint_as_float(s_t2max[j & 3]));
                    if (jn == 0 && lane == 0 && j >= 2) s_t2max[(j - 2) & 3] = 0u;   // read by every Q wave
                    inv2 = __builtin_ldexpf(1.f, -k2);
                }
#pragma unroll
                for (int m = 0; m < 8; ++m) {
                    __builtin_amdgcn_sched_barrier(0);
                    u32x4 tf[2][2];
#pragma unroll
                    for (int s = 0; s < 2; ++s) {
                        const int off = lds_off(16 * m + li, 4 * s + g);
                        tf[s][0] = *(const u32x4*)(lt2 + off);
                        tf[s][1] = *(const u32x4*)(lt2 + T2PL + off);
                    }
                    if (h == 1 && m == 7) post_flag(s_flag + 3, lane);   // t2 read completely
                    f32x4_t acc[2] = {f32x4_t{0.f, 0.f, 0.f, 0.f}, f32x4_t{0.f, 0.f, 0.f, 0.f}};
                    if (!(a.dbg & 4))
#pragma unroll
                        for (int jt = 0; jt < 2; ++jt)
#pragma unroll
                            for (int s = 0; s < 2; ++s) acc[jt] = mfma_pair(w3f[jt][s], tf[s], acc[jt]);
                    int cb = cb0 + 8 * g;
                    asm volatile("" : "+v"(cb));
                    const float4 sa = *(const float4*)(s3 + cb), sb = *(const float4*)(s3 + cb + 4);
                    const float4 ha = *(const float4*)(h3 + cb), hb = *(const float4*)(h3 + cb + 4);
                    const float scv[8] = {sa.x, sa.y, sa.z, sa.w, sb.x, sb.y, sb.z, sb.w};
                    const float shv[8] = {ha.x, ha.y, ha.z, ha.w, hb.x, hb.y, hb.z, hb.w};
                    float v[8];
#pragma unroll
                    for (int e = 0; e < 8; ++e) {
                        v[e] = (acc[e >> 2][e & 3] * inv2) * scv[e] + shv[e] + __uint_as_float(xi[m][e >> 2][e & 3]);
                        v[e] = v[e] > 0.f ? v[e] : 0.f;
                        om_t = fmaxf(om_t, v[e]);
                    }
                    const int oy = oy0 + m;
                    const unsigned so = (oy < a.H && ox < a.W && !(a.dbg & 8)) ? (unsigned)((oy * a.W + ox) * CO + cb) * 4u
                                                                               : 0x80000000u;
                    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, f32x4_t{v[0], v[1], v[2], v[3]}),
                                                           ry, so, 0, 0);
                    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, f32x4_t{v[4], v[5], v[6], v[7]}),
                                                           ry, so, 16, 0);
                }
            }
            om_t = wave_max(om_t);
            if (b != ob) {
                if (ob >= 0 && lane == 0 && om > 0.f) atomicMax(a.ymax + ob, __float_as_uint(om));
                ob = b;
                om = 0.f;
            }
            om = fmaxf(om, om_t);
        }
        if (ob >= 0 && lane == 0 && om > 0.f) atomicMax(a.ymax + ob, __float_as_uint(om));
    }
}

template <int CIN, int XS, int PRE>
hipError_t launch_pipe(const Block32Args& a, hipStream_t s) {
    constexpr size_t lds = (size_t)2 * (CIN / 32) * 4096 + 2 * T1PL + 2 * T2PL + 768 * 4 + 16 * 4;
    static const int cus = [] {
        (void)hipFuncSetAttribute((const void*)bottleneck32p_kernel<CIN, XS, PRE>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)lds);
        int dev = 0, n = 256;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
        return n > 0 ? n : 256;
    }();
    const int tiles = a.B * a.tiles_x * a.tiles_y;
    const int grid = tiles < cus ? tiles : cus;
    hipLaunchKernelGGL((bottleneck32p_kernel<CIN, XS, PRE>), dim3(grid), dim3(768), lds, s, a);
    return hipGetLastError();
}

template <int CIN, bool DS, int XD>
hipError_t launch(const Block32Args& a, hipStream_t s) {
    constexpr size_t lds = (size_t)2 * (CIN / 32) * 4096 + 2 * T1PL + 2 * T2PL + (256 + 512 * (DS ? 2 : 1)) * 4 + 16;
    static const int cus = [] {
        (void)hipFuncSetAttribute((const void*)bottleneck32_kernel<CIN, DS, XD>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        int dev = 0, n = 256;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
        return n > 0 ? n : 256;
    }();
    const int tiles = a.B * a.tiles_x * a.tiles_y;
    const int grid = tiles < cus ? tiles : cus;            // persistent: one workgroup per CU
    hipLaunchKernelGGL((bottleneck32_kernel<CIN, DS, XD>), dim3(grid), dim3(512), lds, s, a);
    return hipGetLastError();
}

}  // namespace

bool vd_block32_ok(int cin, bool ds, int h, int w) {
    if (!((cin == 256 && !ds) || (cin == 64 && ds))) return false;
    return h > 0 && w > 0 && (double)h * w * cin * 4 < 2147483647.0 && (double)h * w * CO * 4 < 2147483647.0;
}

hipError_t vd_launch_block32(const Block32Args& a, hipStream_t s) {
    if (a.B <= 0) return hipSuccess;
    if (!a.xmax || !a.ymax) return hipErrorInvalidValue;
    if (a.cin == 256 && !a.ds) {
        if (a.pipe == 4) return launch_pipe<256, 4, 2>(a, s);   // option block32_pipe: stage-1 x sets
        if (a.pipe == 5) return launch_pipe<256, 5, 2>(a, s);
        if (a.pipe == 6) return launch_pipe<256, 6, 3>(a, s);
        if (a.pipe) return launch_pipe<256, 3, 1>(a, s);
        if (a.xdepth == 3) return launch<256, false, 3>(a, s);
        if (a.xdepth == 4) return launch<256, false, 4>(a, s);
        return launch<256, false, 2>(a, s);
    }
    if (a.cin == 64 && a.ds) return launch<64, true, 2>(a, s);
    return hipErrorInvalidValue;
}
