// chain32.hip — fp32 plan: a layer2 bottleneck's conv3 and the NEXT bottleneck's
// conv1 in one streaming pass (128 -> 512 -> 128 channels).
//
// torchvision Bottleneck [ext] as built from the reference's body.layer2.* weights
// (detect_face/retinaface.py:53-60, IntermediateLayerGetter over resnet50), in the
// arithmetic of the fp32 plan (conv_x6.hip: f32 activations, each product as three
// fp16 MFMA products of power-of-two-scaled hi/lo pairs, f32 accumulation):
//   y   = relu(bn3(conv3(t2)) + idt)        512 ch: this block's output (and the next
//                                            block's identity), written once
//   t1' = relu(bn1'(conv1'(y)))             128 ch: the next block's conv1
// The two-launch plan writes y (840 MB per 64 frames at 80x80) and reads it straight
// back for conv1'; here conv1' consumes it from registers.
//
// One persistent workgroup of 8 waves per CU walks super-groups of 128 pixels, wave w
// taking 16 of them; weights stream through LDS in 8 chunks of 64 conv3 output channels
// (the conv3 rows of the chunk + the conv1' columns that read them: 32 + 32 KB per
// chunk, double-buffered by LDS-DMA with a source-side chunk swizzle):
//   conv3    D^T = W3 . T2^T on 16x16x32 f16 MFMAs (A = weight rows from LDS, B = the
//            wave's 16 pixels, split once per super-group with t2's per-frame scale, as
//            the streaming 1x1 kernel does: y is bit-identical to the two-launch plan);
//            BN + identity + ReLU, 16-B f32 stores of y, per-frame max |y|.
//   conv1'   the lane's y values of conv3 blocks 2i, 2i+1 (channels 32i + 4q + e and
//            32i + 16 + 4q + e of pixel p) are exactly the B fragment of conv1' k-step i
//            once conv1's weights are packed with that K order inside each 32-channel step
//            (Ctx::fuse_chains32). They are split with a per-(pixel, chunk) power of two
//            from the pixel's chunk maximum (two lane shuffles); the pixel's running sum
//            is kept at the current chunk's scale (re-based by an exact power-of-two
//            multiply when the scale changes), so all of conv1's K accumulates in one
//            chain as in the two-launch plan, only the split points differ: f32-level
//            differences (tests/test_gpu_e2e.py), batch-invariant (nothing depends on
//            the pixel's neighbours in the batch).
// vmcnt counts LDS-DMA, loads and stores together in issue order; every wave issues the
// same count of each per chunk (8 DMA, 4 identity loads, 4 y stores), so the waits are
// fixed immediates.
#include "vd_common.h"

namespace {

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 half2_t __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) void lds_void_t;

// Shapes: layer2 (t2 128 -> y 512 -> t1' 128; weight chunks of 64 conv3 channels) and
// layer3 (256 -> 1024 -> 256; chunks of 32). Either way a chunk is 32 KB of W3 rows and
// 32 KB of W1 columns, and a wave runs 48 + 48 MFMAs on it.
template <int CM_, int CO_, int NCH_, int GPW_, int WAVES_ = 8> struct ChainShape {
    static constexpr int CM = CM_, CO = CO_, NCH = NCH_;
    static constexpr int GPW = GPW_;             // 16-pixel groups per wave
    static constexpr int WAVES = WAVES_;
    static constexpr int SGG = GPW * WAVES;      // groups per super-group (one pass of the weights)
    static constexpr int THREADS = 64 * WAVES;
    static constexpr int ND = 64 / WAVES;        // weight DMA instructions per wave per chunk
    static constexpr int KS3 = CM / 32;          // conv3 k-steps
    static constexpr int T3 = NCH / 16;          // conv3 tiles per chunk
    static constexpr int KC = NCH / 32;          // conv1' k-steps per chunk
    static constexpr int T1 = CM / 16;           // conv1' output tiles
    static constexpr int NCHUNK = CO / NCH;
    static constexpr int RB3 = KS3 * 128;        // W3 row bytes (k-steps x 2 planes x 64 B)
    static constexpr int RB1 = KC * 128;         // W1 row slice bytes of one chunk
    static constexpr int W3B = NCH * RB3, W1B = CM * RB1, STAGE = W3B + W1B;
    static constexpr int LDS = 2 * STAGE + (2 * CO + 2 * CM) * 4;
    static_assert(W3B == 32768 && W1B == 32768, "64-KB stages");
};
using L2Shape = ChainShape<128, 512, 64, 1>;    // 8 waves of 16 pixels: 128-pixel super-groups
using L2Shape2 = ChainShape<128, 512, 64, 2>;   // option chain_gpw=2: 32 pixels per wave (~55 VGPRs spill)
using L3Shape = ChainShape<256, 1024, 32, 1>;

// s_waitcnt vmcnt(N), expcnt / lgkmcnt left alone (gfx9 encoding)
constexpr int vmcnt_imm(int n) { return (n & 15) | ((n >> 4) << 14) | 0x0F70; }

__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// 8 f32 -> fp16 hi / lo planes of x * sa (conv_x6.hip split_pair8: the same roundings)
__device__ __forceinline__ void split8(const float (&e)[8], float sa, u32x4& H, u32x4& L) {
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

// w_lo x_hi + w_hi x_lo + w_hi x_hi (conv_x6.hip mfma_terms<2>, small terms first)
__device__ __forceinline__ f32x4_t mfma3(const u32x4& wh, const u32x4& wl, const u32x4& xh, const u32x4& xl,
                                         f32x4_t acc) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8_t, wl), __builtin_bit_cast(f16x8_t, xh), acc,
                                                 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8_t, wh), __builtin_bit_cast(f16x8_t, xl), acc,
                                                 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8_t, wh), __builtin_bit_cast(f16x8_t, xh), acc,
                                                 0, 0, 0);
    return acc;
}

// power-of-two exponent k with m * 2^k in [2^14, 2^15) (act_scale_exp's rule)
__device__ __forceinline__ int pow2_exp(float m) {
    if (!(m > 0.f) || !(m < 3.0e38f)) return 0;
    int e;
    (void)frexpf(m, &e);
    const int k = 15 - e;
    return k < -100 ? -100 : (k > 100 ? 100 : k);
}

template <class S>
__global__ __launch_bounds__(S::THREADS, 1) void chain32_kernel(Chain32Args a) {
    constexpr int CM = S::CM, CO = S::CO, NCH = S::NCH, KS3 = S::KS3, T3 = S::T3, KC = S::KC, T1 = S::T1;
    constexpr int NCHUNK = S::NCHUNK, RB3 = S::RB3, RB1 = S::RB1, W3B = S::W3B, STAGE = S::STAGE;
    constexpr int GPW = S::GPW, NT = S::THREADS, ND = S::ND;
    // LDS row -> swizzle key: 16-B chunk ci of a row sits at ci ^ key (conflict-free
    // fragment reads of 16 consecutive rows; rows of 128 B pair up in a 256-B bank line)
    constexpr int R1PL = 256 / (RB1 < 256 ? RB1 : 256), C1 = RB1 / 16;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    float* s_sc3 = (float*)(smem + 2 * STAGE);
    float* s_sh3 = s_sc3 + CO;
    float* s_sc1 = s_sh3 + CO;
    float* s_sh1 = s_sc1 + CM;
    unsigned* s_ymax = (unsigned*)(s_sh1 + CM);            // [B] then [B]
    unsigned* s_y2max = s_ymax + a.B;

    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int p = lane & 15, q = lane >> 4;
    constexpr int SGG = S::SGG;
    const int nsg = (a.M + 16 * SGG - 1) / (16 * SGG);
    const int G = gridDim.x, sg0 = blockIdx.x;
    if (sg0 >= nsg) return;                                 // uniform over the workgroup
    const int nmine = (nsg - sg0 + G - 1) / G;

    for (int i = tid; i < CO; i += NT) { s_sc3[i] = a.sc3[i]; s_sh3[i] = a.sh3[i]; }
    for (int i = tid; i < CM; i += NT) { s_sc1[i] = a.sc1[i]; s_sh1[i] = a.sh1[i]; }
    for (int f = tid; f < 2 * a.B; f += NT) s_ymax[f] = 0u;

    const __amdgpu_buffer_rsrc_t rw3 = __builtin_amdgcn_make_buffer_rsrc((void*)a.w3, 0, 0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t rw1 = __builtin_amdgcn_make_buffer_rsrc((void*)a.w1, 0, 0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc((void*)a.t2, 0, 0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc((void*)a.res, 0, 0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t ry =
        __builtin_amdgcn_make_buffer_rsrc(a.y, 0, (int)((long)a.M * a.ld_y * 4), 0x00020000);
    const __amdgpu_buffer_rsrc_t ry2 =
        __builtin_amdgcn_make_buffer_rsrc(a.y2, 0, (int)((long)a.M * a.ld_y2 * 4), 0x00020000);

    // DMA of weight chunk c into stage st: 64 instructions of 1 KB, ND per wave
    // (instructions 0-31: the chunk's W3 rows NCH c .. +NCH; 32-63: the RB1-byte slice
    // [RB1 c, RB1 (c + 1)) of each of the CM W1 rows). LDS position pos of a row holds
    // logical 16-B chunk pos ^ key(row).
    auto dma = [&](int c, int st) {
        char* base = smem + st * STAGE;
#pragma unroll
        for (int u = 0; u < ND; ++u) {
            const int k = w * ND + u;
            if (k < 32) {
                constexpr int RPI = 1024 / RB3;             // rows per instruction
                const int r = RPI * k + lane / (64 / RPI), pos = lane % (64 / RPI);
                const int ci = pos ^ (r & 15);
                const unsigned off = (unsigned)((NCH * c + r) * RB3 + ci * 16);
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rw3, (lds_void_t*)(base + k * 1024), 16, off, 0, 0, 0);
            } else {
                constexpr int RPI = 1024 / RB1;
                const int kk = k - 32;
                const int r = RPI * kk + lane / C1, pos = lane % C1;
                const int ci = pos ^ ((r / R1PL) & (C1 - 1));
                const unsigned off = (unsigned)(r * (CO / 32) * 128 + c * RB1 + ci * 16);
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rw1, (lds_void_t*)(base + W3B + kk * 1024), 16, off, 0, 0, 0);
            }
        }
    };
    // this lane's pixel of 16-pixel group g (clamped; stores past M are dropped by ry / ry2)
    auto pixel = [&](int g) {
        const int m = g * 16 + p;
        return m < a.M ? m : a.M - 1;
    };
    auto load_x = [&](int g, u32x4 (&xr)[KS3][2]) {
        const unsigned base = (unsigned)(pixel(g) * a.ld_t2 + 8 * q) * 4u;
#pragma unroll
        for (int s = 0; s < KS3; ++s) {
            xr[s][0] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rx, (int)(base + 128u * s), 0, 0));
            xr[s][1] =
                __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rx, (int)(base + 128u * s + 16u), 0, 0));
        }
    };
    // identity of chunk c: channels NCH c + 16j + 4q .. +3, j < T3
    auto load_idt = [&](int g, int c, u32x4 (&r)[T3]) {
        const unsigned base = (unsigned)(pixel(g) * a.ld_res + NCH * c + 4 * q) * 4u;
#pragma unroll
        for (int j = 0; j < T3; ++j)
            r[j] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rr, (int)(base + 64u * j), 0, 0));
    };

    // wave w takes groups GPW w .. +GPW of each super-group of SGG groups
    int g0 = sg0 * SGG + GPW * w;
    // IDB: the identity of chunk c + 1 loaded during chunk c (two register sets); with two
    // groups per wave there is room for one set only, loaded at the top of its own chunk
    constexpr bool IDB = GPW == 1;
    u32x4 xr[GPW][KS3][2], idt[IDB ? 2 : 1][GPW][T3];
    dma(0, 0);
    if constexpr (IDB) {
#pragma unroll
        for (int u = 0; u < GPW; ++u) load_idt(g0 + u, 0, idt[0][u]);
    }
#pragma unroll 1
    for (int it = 0; it < nmine; ++it) {
        const int gn = it + 1 < nmine ? (sg0 + (it + 1) * G) * SGG + GPW * w : g0;   // next super-group
        // x of this super-group (GPW = 1: loaded at the end of the previous one)
        if (GPW > 1 || it == 0) {
#pragma unroll
            for (int u = 0; u < GPW; ++u) load_x(g0 + u, xr[u]);
        }
        __builtin_amdgcn_s_waitcnt(vmcnt_imm(0));          // x, identity(0), weight chunk 0
        int m[GPW], fb[GPW];
        bool ok[GPW];
        float inv_sa[GPW];
        u32x4 xb[GPW][KS3][2];
#pragma unroll
        for (int u = 0; u < GPW; ++u) {
            m[u] = (g0 + u) * 16 + p;
            ok[u] = m[u] < a.M;
            fb[u] = (ok[u] ? m[u] : a.M - 1) / a.hw;        // this lane's pixel's frame
            const float mx = a.xmax ? __uint_as_float(a.xmax[fb[u]]) : a.xbound;
            const int kx = pow2_exp(mx);
            const float sa = __builtin_ldexpf(1.f, kx);
            inv_sa[u] = __builtin_ldexpf(1.f, -kx);
#pragma unroll
            for (int s = 0; s < KS3; ++s) {
                float e8[8];
#pragma unroll
                for (int e = 0; e < 8; ++e) e8[e] = __uint_as_float(xr[u][s][e >> 2][e & 3]);
                split8(e8, sa, xb[u][s][0], xb[u][s][1]);
            }
        }
        f32x4_t acc1[GPW][T1];
#pragma unroll
        for (int u = 0; u < GPW; ++u)
#pragma unroll
            for (int j = 0; j < T1; ++j) acc1[u][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
        float vmax_y[GPW];
        int ks[GPW];                                        // scale exponent of acc1
#pragma unroll
        for (int u = 0; u < GPW; ++u) { vmax_y[u] = 0.f; ks[u] = 0; }
#pragma unroll 1
        for (int cp = 0; cp < NCHUNK / 2; ++cp)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int c = 2 * cp + h, st = h;               // chunk c in stage c & 1
            // chunk c landed (younger: identity(c) when prefetched, y(c-1))
            if (c > 0) __builtin_amdgcn_s_waitcnt(vmcnt_imm((IDB ? 2 : 1) * GPW * T3));
            lds_barrier();                                  // every wave's DMA of chunk c landed; stage st^1 free
            const int cn = c + 1 < NCHUNK ? c + 1 : 0;
            if constexpr (!IDB) {
#pragma unroll
                for (int u = 0; u < GPW; ++u) load_idt(g0 + u, c, idt[0][u]);
            }
            dma(cn, st ^ 1);
            if constexpr (IDB) {
#pragma unroll
                for (int u = 0; u < GPW; ++u) load_idt((cn == 0 ? gn : g0) + u, cn, idt[h ^ 1][u]);
            }
            const char* w3s = smem + st * STAGE;
            const char* w1s = w3s + W3B;
            // ---- conv3, channels NCH c .. +NCH of the wave's pixels ----
            f32x4_t acc3[GPW][T3];
#pragma unroll
            for (int u = 0; u < GPW; ++u)
#pragma unroll
                for (int j = 0; j < T3; ++j) acc3[u][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int s = 0; s < KS3; ++s) {
#pragma unroll
                for (int j = 0; j < T3; ++j) {
                    const char* row = w3s + (16 * j + p) * RB3;
                    const u32x4 wh = *(const u32x4*)(row + ((((2 * s) * 4 + q) ^ p) << 4));
                    const u32x4 wl = *(const u32x4*)(row + ((((2 * s + 1) * 4 + q) ^ p) << 4));
#pragma unroll
                    for (int u = 0; u < GPW; ++u) acc3[u][j] = mfma3(wh, wl, xb[u][s][0], xb[u][s][1], acc3[u][j]);
                }
                // GPW = 2: keep each k-step's fragment reads next to its MFMAs (read ahead,
                // the whole chunk's fragments would need another 128 VGPRs)
                if constexpr (GPW > 1 || KS3 > 4) __builtin_amdgcn_sched_barrier(0);
            }
            // ---- epilogue: bn3 + identity + relu, store y, split for conv1' ----
            // identity(c) (younger: y(c-1), DMA(c+1), identity(c+1))
            // IDB: younger than identity(c) are y(c-1), DMA(c+1), identity(c+1); else DMA(c+1)
            __builtin_amdgcn_s_waitcnt(vmcnt_imm(IDB ? ND + 2 * GPW * T3 : ND));
            u32x4 yb[GPW][KC][2];
#pragma unroll
            for (int u = 0; u < GPW; ++u) {
                float yv[T3][4];
                float cmax = 0.f;
                const unsigned ybase = ok[u] ? (unsigned)(m[u] * a.ld_y + NCH * c + 4 * q) * 4u : 0x80000000u;
#pragma unroll
                for (int j = 0; j < T3; ++j) {
                    const int ch = NCH * c + 16 * j + 4 * q;
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const float v = (acc3[u][j][e] * inv_sa[u]) * s_sc3[ch + e] + s_sh3[ch + e];
                        float t = v + __uint_as_float(idt[IDB ? h : 0][u][j][e]);
                        t = t > 0.f ? t : 0.f;
                        yv[j][e] = t;
                        cmax = fmaxf(cmax, t);
                    }
                    __builtin_amdgcn_raw_buffer_store_b128(
                        __builtin_bit_cast(u32x4, f32x4_t{yv[j][0], yv[j][1], yv[j][2], yv[j][3]}), ry,
                        (int)(ybase + (ok[u] ? 64u * j : 0u)), 0, 0);
                }
                vmax_y[u] = fmaxf(vmax_y[u], cmax);
                cmax = fmaxf(cmax, __shfl_xor(cmax, 16));
                cmax = fmaxf(cmax, __shfl_xor(cmax, 32));   // the pixel's max over the chunk's NCH channels
                // the pixel's conv1' sum runs at scale 2^ks: re-based exactly (a power of
                // two) when this chunk's split scale differs; an all-zero chunk keeps it
                const int ky = cmax > 0.f ? pow2_exp(cmax) : ks[u];
                const float rebase = __builtin_ldexpf(1.f, ky - ks[u]);
                ks[u] = ky;
                const float sy = __builtin_ldexpf(1.f, ky);
#pragma unroll
                for (int j = 0; j < T1; ++j)
#pragma unroll
                    for (int e = 0; e < 4; ++e) acc1[u][j][e] *= rebase;
#pragma unroll
                for (int i = 0; i < KC; ++i) {
                    const float e8[8] = {yv[2 * i][0], yv[2 * i][1], yv[2 * i][2], yv[2 * i][3],
                                         yv[2 * i + 1][0], yv[2 * i + 1][1], yv[2 * i + 1][2], yv[2 * i + 1][3]};
                    split8(e8, sy, yb[u][i][0], yb[u][i][1]);
                }
            }
            // ---- conv1' over the chunk's NCH input channels, into the running sums ----
#pragma unroll
            for (int i = 0; i < KC; ++i) {
#pragma unroll
                for (int j = 0; j < T1; ++j) {
                    const int r = 16 * j + p, key = (r / R1PL) & (C1 - 1);
                    const char* row = w1s + r * RB1;
                    const u32x4 wh = *(const u32x4*)(row + ((((2 * i) * 4 + q) ^ key) << 4));
                    const u32x4 wl = *(const u32x4*)(row + ((((2 * i + 1) * 4 + q) ^ key) << 4));
#pragma unroll
                    for (int u = 0; u < GPW; ++u) acc1[u][j] = mfma3(wh, wl, yb[u][i][0], yb[u][i][1], acc1[u][j]);
                    if constexpr (GPW > 1 || T1 > 8) {
                        if ((j & 1) == 1) __builtin_amdgcn_sched_barrier(0);
                    }
                }
            }
        }
        // ---- conv1' epilogue: bn1' + relu, t1' stores ----
#pragma unroll
        for (int u = 0; u < GPW; ++u) {
            const float inv_s1 = __builtin_ldexpf(1.f, -ks[u]);
            float vmax_t = 0.f;
            const unsigned y2base = ok[u] ? (unsigned)(m[u] * a.ld_y2 + 4 * q) * 4u : 0x80000000u;
#pragma unroll
            for (int j = 0; j < T1; ++j) {
                float o[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int ch = 16 * j + 4 * q + e;
                    const float t = (acc1[u][j][e] * inv_s1) * s_sc1[ch] + s_sh1[ch];
                    o[e] = t > 0.f ? t : 0.f;
                    vmax_t = fmaxf(vmax_t, o[e]);
                }
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, f32x4_t{o[0], o[1], o[2], o[3]}), ry2,
                                                       (int)(y2base + (ok[u] ? 64u * j : 0u)), 0, 0);
            }
            amax_lds_add(s_ymax, ok[u] ? fb[u] : -1, vmax_y[u]);
            amax_lds_add(s_y2max, ok[u] ? fb[u] : -1, vmax_t);
        }
        g0 = gn;
        if constexpr (GPW == 1) load_x(g0, xr[0]);
    }
    __builtin_amdgcn_s_waitcnt(vmcnt_imm(0));               // trailing DMA / loads land before the workgroup exits
    __syncthreads();
    if (a.ymax) amax_lds_flush(s_ymax, a.ymax, a.B);
    if (a.y2max) amax_lds_flush(s_y2max, a.y2max, a.B);
}

}  // namespace

// Eligible: the layer2 (128 -> 512 -> 128) or layer3 (256 -> 1024 -> 256) shape with
// dense rows, frames within the LDS max slots, byte offsets within 2^31.
bool vd_chain32_ok(int cmid, int cout, int kpad3, int kpad1, int ld_t2, int ld_res, int ld_y, int ld_y2, long M,
                   int frames) {
    const bool l2 = cmid == 128 && cout == 512, l3 = cmid == 256 && cout == 1024;
    if (!(l2 || l3) || kpad3 != cmid || kpad1 != cout) return false;
    if (ld_t2 != cmid || ld_res != cout || ld_y != cout || ld_y2 != cmid) return false;
    return M > 0 && M * cout * 4 < 0x7fffffffL && frames > 0 && frames <= 1024;
}

template <class S>
static hipError_t launch_chain32_t(const Chain32Args& a, hipStream_t s) {
    static const int cus = [] {
        (void)hipFuncSetAttribute((const void*)chain32_kernel<S>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  S::LDS + 8 * 1024);
        int dev = 0, n = 256;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
        return n > 0 ? n : 256;
    }();
    const int nsg = (a.M + 16 * S::SGG - 1) / (16 * S::SGG);
    const int grid = nsg < cus ? nsg : cus;                 // persistent: one workgroup per CU
    hipLaunchKernelGGL(chain32_kernel<S>, dim3(grid), dim3(S::THREADS), S::LDS + 8 * a.B, s, a);
    return hipGetLastError();
}

hipError_t vd_launch_chain32(const Chain32Args& a, hipStream_t s) {
    if (a.M <= 0) return hipSuccess;
    if (a.B <= 0 || a.B > 1024 || a.hw <= 0) return hipErrorInvalidValue;
    if (a.ld_t2 == 128 && a.ld_res == 512)
        return a.gpw == 2 ? launch_chain32_t<L2Shape2>(a, s) : launch_chain32_t<L2Shape>(a, s);
    if (a.ld_t2 == 256 && a.ld_res == 1024) return launch_chain32_t<L3Shape>(a, s);
    return hipErrorInvalidValue;
}
