// block.hip — one whole ResNet-50 layer1 bottleneck in one kernel.
//
// torchvision Bottleneck [ext] (torchvision/models/resnet.py, v1.5) as built
// from the reference's body.layer1.* weights (detect_face/retinaface.py:53-60,
// IntermediateLayerGetter over resnet50):
//   t1  = relu(bn1(conv1x1(x)))            64 ch, on the 10x18 halo of the tile
//   t2  = relu(bn2(conv3x3(t1, pad 1)))    64 ch
//   out = relu(bn3(conv1x1(t2)) + idt)     256 ch; idt = x (layer1.1, layer1.2) or
//                                          bn(downsample(x)) (layer1.0, CIN = 64)
// Same arithmetic contract as the per-conv kernels (bf16 operands, f32
// accumulation, BN as acc*scale + shift, t1/t2 rounded to bf16), but t1 and t2
// never leave LDS: per output pixel HBM sees x once and out once (1 KB) instead of
// the ~2 KB of the conv-by-conv chain, and the four launches become one.
//
// One workgroup = one 8x16-pixel output tile of one frame, 4 waves:
//   stage 1  D^T = W1 . X^T over the 180 halo pixels (12 MFMA row tiles, 3 per wave),
//            X fragments straight from HBM (zero past the frame through buffer
//            loads), W1 from LDS; BN+ReLU -> t1 in LDS (zero outside the frame = the
//            3x3 conv's padding).
//   stage 2  wave w computes t2 channels 16w..16w+15 for all 128 pixels: its W2
//            fragments (16 x 576) sit in VGPRs, the shifted t1 windows come from LDS.
//   stage 3  wave w computes out channels 64w..64w+63 (W3, and Wd, fragments in
//            VGPRs), one 16-pixel output row at a time; residual / BN / ReLU in
//            registers, 16-B stores of 8 consecutive channels per lane.
// LDS: W1 image (CIN x 64) + t1 (192 x 64) + t2 (128 x 64) bf16 + BN tables, 54-75 KB:
// two workgroups per CU, so one tile's loads overlap the other's MFMAs.
#include "vd_common.h"

#include <cstdlib>

namespace {

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

constexpr int TH = 8, TW = 16;                  // output tile
constexpr int HWD = TW + 2;                     // halo width
constexpr int HROWS = (TH + 2) * HWD;           // 180 halo pixels
constexpr int P = 64, CO = 256;                 // bottleneck width, output channels

// t1 / t2 images: 128-B rows of 64 channels, 16-B chunk c of row r at chunk
// c ^ (2 * ((r >> 1) & 3)). Conflict-free ds_read_b128 for ANY 16 consecutive rows
// (stage 2 reads windows shifted by the tap offsets): each 16-lane LDS group holds
// all 16 rows once, 8 of them at chunk c and 8 at c ^ 1 in a cyclic block of 4 row
// pairs, and this XOR keeps the 8 even (and the 8 odd) rows on distinct 16-B slots
// for every block position (exhaustive check; the (r >> 1) & 7 swizzle is 2-way here)
__device__ __forceinline__ int lds_off(int row, int chunk) {
    return row * 128 + ((chunk ^ (((row >> 1) & 3) << 1)) << 4);
}

typedef __attribute__((address_space(3))) void lds_void_t;

// physical 16-B chunk of logical chunk c in row r of the x halo image: 512-B rows
// (CIN 256) XOR the low 4 chunk bits with r&15, 128-B rows (CIN 64) with (r>>1)&7 --
// conflict-free ds_read_b128 for 16 consecutive rows at one chunk
template <int CIN>
__device__ __forceinline__ int lx_chunk(int r, int c) {
    if constexpr (CIN == 256) return c ^ (r & 15);
    else return c ^ ((r >> 1) & 7);
}

constexpr int VMCNT0 = 0x0F70;                  // s_waitcnt vmcnt(0) (expcnt / lgkmcnt: no wait)
constexpr int VMCNT8 = 0x0F78;                  // s_waitcnt vmcnt(8)

// F16: the fp16 plan (VD_PREC_FP16) -- the same kernel on fp16 operands / activations
template <int CIN, bool DS, bool F16>
__global__ __launch_bounds__(512, 1) void bottleneck_kernel(BlockArgs a) {
    using HT = Half16<F16>;
    typedef typename HT::T E16;
    typedef E16 t16x4_t __attribute__((ext_vector_type(4)));
    const auto mfma = [](const u32x4& x, const u32x4& y, const f32x4_t& c) { return HT::mfma(x, y, c); };
    constexpr int KS1 = CIN / 32;                         // stage-1 k-steps
    constexpr int XROW = CIN * 2;                         // bytes per halo pixel in LX
    constexpr int RPI = 1024 / XROW;                      // pixels per 1-KB DMA instruction
    constexpr int XROWS = (HROWS + RPI - 1) / RPI * RPI;  // 180 (CIN 256) / 184 (CIN 64)
    constexpr int NDMA = XROWS / RPI;
    constexpr int XB = XROWS * XROW;
    constexpr int NXB = DS ? 2 : 1;                       // DS reads x again in stage 3: double buffer
    constexpr int DPW = (NDMA + 7) / 8;                   // DMA instructions per wave per tile
    constexpr bool W1_STAT = KS1 <= 2;                    // W1 in VGPRs for good (CIN 64) or reloaded per tile
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* lx = smem;
    char* lt1 = lx + NXB * XB;
    char* lt2 = lt1 + 192 * 128;
    char* lscratch = lt2 + 128 * 128;                     // sink of the padding DMA slots (1 KB)

    const int tid = threadIdx.x, lane = tid & 63, li0 = lane & 15, g0 = lane >> 4;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform (SGPR) from here on
    const int jn = w & 3, half = w >> 2;
    const int tpf = a.tiles_x * a.tiles_y, T = a.B * tpf;
    // tiles of this workgroup: each XCD takes a contiguous range (halo neighbours share its L2)
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
    const size_t fpx = (size_t)a.H * a.W;

    // x halo tile of tile t -> LX buffer: one 1-KB buffer_load...lds per RPI pixels,
    // chunk-swizzled through the source addresses (the DMA writes lane-linear)
    auto issue_x = [&](int t, int buf) {
        const int b = t / tpf, r0 = t - b * tpf;
        const int ty = r0 / a.tiles_x, tx = r0 - ty * a.tiles_x;
        const int oy0 = ty * TH, ox0 = tx * TW;
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            (void*)((const E16*)a.x + (size_t)b * fpx * CIN), 0, (int)(fpx * CIN * 2), 0x00020000);
        // every wave issues exactly DPW DMAs (slots past NDMA read zeros into a 1-KB
        // scratch line): a compile-time count keeps the compiler's vmcnt bookkeeping
        // exact, so later waits on W2 / residual loads do not also wait for this DMA
        char* dst = lx + buf * XB;
#pragma unroll
        for (int k = 0; k < DPW; ++k) {
            const int i = w + 8 * k;
            const bool real = i < NDMA;
            const int r = i * RPI + lane / (64 / RPI);
            const int cp = lane % (64 / RPI);
            const int c = lx_chunk<CIN>(r, cp);
            const int hy = r / HWD, hx = r - hy * HWD;
            const int iy = oy0 - 1 + hy, ix = ox0 - 1 + hx;
            const bool in = real && r < HROWS && (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W;
            const unsigned off = in ? (unsigned)((iy * a.W + ix) * XROW + c * 16) : 0x80000000u;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void_t*)(real ? dst + i * 1024 : lscratch), 16, off, 0,
                                                     0, 0);
        }
    };
    issue_x(t0, 0);

    // per-lane BN constants: stages 1/2 own channels 16jn + 4g + (0..3), stage 3
    // channels 32w + 8g + (0..7)
    const float4 s1v = *(const float4*)(a.bn + 16 * jn + 4 * g0), h1v = *(const float4*)(a.bn + 64 + 16 * jn + 4 * g0);
    const float4 s2v = *(const float4*)(a.bn + 128 + 16 * jn + 4 * g0), h2v = *(const float4*)(a.bn + 192 + 16 * jn + 4 * g0);
    float s3[8], h3[8], sd[DS ? 8 : 1], hd[DS ? 8 : 1];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        s3[e] = a.bn[256 + 32 * w + 8 * g0 + e];
        h3[e] = a.bn[512 + 32 * w + 8 * g0 + e];
        if constexpr (DS) {
            sd[e] = a.bn[768 + 32 * w + 8 * g0 + e];
            hd[e] = a.bn[1024 + 32 * w + 8 * g0 + e];
        }
    }
    // weight fragments: W1 (this wave's 16 channels; reloaded per tile during stage 3),
    // W3 / Wd (its 32 channels; stationary)
    // weight fragments through buffer descriptors: one lane offset (lane * 16 B) and a
    // scalar offset per fragment, so no per-fragment 64-bit addresses live in VGPRs
    const __amdgpu_buffer_rsrc_t rw1 = __builtin_amdgcn_make_buffer_rsrc((void*)a.w1, 0, 0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t rw2 = __builtin_amdgcn_make_buffer_rsrc((void*)a.w2, 0, 0x7fffffff, 0x00020000);
    const unsigned lo16 = (unsigned)lane * 16u;
    // stationary for the workgroup's life: W2 (this wave's 16 channels), W3 / Wd (its 32
    // channels), and W1 when CIN = 64 -- per-tile reloads of W2 alone would move 144 KB
    // per tile through the CU's load path. W1 at CIN = 256 (32 VGPRs) is reloaded per tile.
    u32x4 w1f[KS1], w2f[18], w3f[2][2], wdf[DS ? 2 : 1][DS ? KS1 : 1];
#pragma unroll
    for (int s = 0; s < KS1; ++s) w1f[s] = __builtin_amdgcn_raw_buffer_load_b128(rw1, lo16, (jn * KS1 + s) * 1024, 0);
#pragma unroll
    for (int s = 0; s < 18; ++s) w2f[s] = __builtin_amdgcn_raw_buffer_load_b128(rw2, lo16, (jn * 18 + s) * 1024, 0);
    {
        const __amdgpu_buffer_rsrc_t rw3 = __builtin_amdgcn_make_buffer_rsrc((void*)a.w3, 0, 0x7fffffff, 0x00020000);
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int s = 0; s < 2; ++s)
                w3f[j][s] = __builtin_amdgcn_raw_buffer_load_b128(rw3, lo16, (w * 4 + j * 2 + s) * 1024, 0);
        if constexpr (DS) {
            const __amdgpu_buffer_rsrc_t rwd = __builtin_amdgcn_make_buffer_rsrc((void*)a.wd, 0, 0x7fffffff, 0x00020000);
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int s = 0; s < KS1; ++s)
                    wdf[j][s] = __builtin_amdgcn_raw_buffer_load_b128(rwd, lo16, ((w * 2 + j) * KS1 + s) * 1024, 0);
        }
    }

    // diagnostics (build with -DVD_BLOCK_DIAG): cycle sums per segment (workgroup 0, wave 0)
#ifdef VD_BLOCK_DIAG
    const bool dg = a.diag != nullptr && bid == 0 && w == 0;
#else
    constexpr bool dg = false;
#endif
    unsigned long long dsum[8] = {0, 0, 0, 0, 0, 0, 0, 0}, dlast = dg ? __builtin_readcyclecounter() : 0;
#define VD_STAMP(I)                                                                                \
    do {                                                                                           \
        if (dg) {                                                                                  \
            const unsigned long long now_ = __builtin_readcyclecounter();                          \
            dsum[I] += now_ - dlast;                                                               \
            dlast = now_;                                                                          \
        }                                                                                          \
    } while (0)
    int buf = 0;
#pragma unroll 1
    for (int t = t0; t < tend; t += tstep) {
        const int b = t / tpf, r0 = t - b * tpf;
        const int ty = r0 / a.tiles_x, tx = r0 - ty * a.tiles_x;
        const int oy0 = ty * TH, ox0 = tx * TW;
        const char* lxc = lx + buf * XB;
        VD_STAMP(7);
        // this tile's x (and all earlier loads). NOTE on vmcnt: the compiler does not count
        // LDS-DMA in its s_waitcnt bookkeeping while the hardware retires VMEM loads in
        // order, so no register load may be consumed while a DMA is in flight -- hence
        // the builtin waits (visible to the compiler) and the load placement below.
        // vmcnt counts loads, stores and LDS-DMA together in issue order: the previous
        // tile's 8 output stores per thread are the only ops younger than this tile's x
        // DMA (and the W1 reload), so vmcnt(8) has them landed without waiting for the stores
        __builtin_amdgcn_s_waitcnt(VMCNT8);
        VD_STAMP(0);
        __syncthreads();
        VD_STAMP(1);
        // lane coordinates made opaque per tile: keeps the ~130 per-lane LDS addresses
        // of the three stages from being hoisted out of the tile loop into VGPRs
        int li = li0, g = g0;
        asm volatile("" : "+v"(li), "+v"(g));

        // ---- stage 1: t1^T (channels 16jn..) over halo row tiles half, half+2, ... ----
        {
            f32x4_t acc[6];
#pragma unroll
            for (int k = 0; k < 6; ++k) acc[k] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int s = 0; s < KS1; ++s) {
                asm volatile("" ::: "memory");
                u32x4 xf[6];
#pragma unroll
                for (int k = 0; k < 6; ++k) {
                    const int r = 16 * (half + 2 * k) + li;
                    xf[k] = *(const u32x4*)(lxc + r * XROW + (lx_chunk<CIN>(r, 4 * s + g) << 4));
                }
#pragma unroll
                for (int k = 0; k < 6; ++k) acc[k] = mfma(w1f[s], xf[k], acc[k]);
            }
#pragma unroll
            for (int k = 0; k < 6; ++k) {
                const int r = 16 * (half + 2 * k) + li;
                const int hy = r / HWD, hx = r - hy * HWD;
                const int iy = oy0 - 1 + hy, ix = ox0 - 1 + hx;
                const bool in = r < HROWS && (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W;
                const float v0 = acc[k][0] * s1v.x + h1v.x, v1 = acc[k][1] * s1v.y + h1v.y;
                const float v2 = acc[k][2] * s1v.z + h1v.z, v3 = acc[k][3] * s1v.w + h1v.w;
                const t16x4_t o = {(E16)(in && v0 > 0.f ? v0 : 0.f), (E16)(in && v1 > 0.f ? v1 : 0.f),
                                   (E16)(in && v2 > 0.f ? v2 : 0.f), (E16)(in && v3 > 0.f ? v3 : 0.f)};
                *(t16x4_t*)(lt1 + lds_off(r, 2 * jn + (g >> 1)) + (g & 1) * 8) = o;
            }
        }
        // the stage-3 identity, x at this wave's 32 channels for the 8 tile rows, taken
        // from the halo image before the next tile's DMA overwrites it (LDS, not the
        // load path; pixels past the frame are zeros there)
        u32x4 rf[DS ? 1 : 8];
        if constexpr (!DS) {
#pragma unroll
            for (int m = 0; m < 8; ++m) {
                const int r = (m + 1) * HWD + li + 1;
                rf[m] = *(const u32x4*)(lxc + r * XROW + (lx_chunk<CIN>(r, 4 * w + g) << 4));
            }
        }
        VD_STAMP(2);
        __syncthreads();   // t1 complete; LX[buf] read for the last time (identity variant)
        VD_STAMP(3);

        // next tile's x into LX (the other buffer when stage 3 still reads this one).
        // No register load is pending here in steady state (weights stationary, the
        // identity from LDS); in the first tile the compiler's waits on the weight
        // loads, blind to the DMA, can only wait longer than needed.
        if (!(a.mode & 1) && t + tstep < tend) issue_x(t + tstep, DS ? buf ^ 1 : 0);

        // ---- stage 2: t2^T (channels 16jn..) over tile rows 4*half .. 4*half+3 ----
        {
            f32x4_t acc[4];
#pragma unroll
            for (int m = 0; m < 4; ++m) acc[m] = f32x4_t{0.f, 0.f, 0.f, 0.f};
            // Each t1 window (halo row 4*half + hh, shift dx, channel half hf) is read once
            // and feeds every output row it touches (m = hh - dy for the three kernel rows
            // dy): 36 reads for the 72 MFMAs. Reads run 3 windows ahead of their MFMAs.
            constexpr int PD = 3;
            u32x4 tf[PD + 1];
#define VD_T1READ(Q)                                                                               \
            do {                                                                                   \
                const int hh_ = (Q) / 6, hf_ = ((Q) / 3) & 1, dx_ = (Q) % 3;                       \
                tf[(Q) % (PD + 1)] = *(const u32x4*)(lt1 + lds_off((4 * half + hh_) * HWD + li + dx_, 4 * hf_ + g)); \
            } while (0)
#pragma unroll
            for (int q = 0; q < PD; ++q) VD_T1READ(q);
#pragma unroll
            for (int q = 0; q < 36; ++q) {
                asm volatile("" ::: "memory");
                if (q + PD < 36) VD_T1READ(q + PD);
                const int hh = q / 6, hf = (q / 3) & 1, dx = q % 3;
#pragma unroll
                for (int dy = 0; dy < 3; ++dy) {
                    const int m = hh - dy;
                    if (m >= 0 && m < 4) acc[m] = mfma(w2f[2 * (3 * dy + dx) + hf], tf[q % (PD + 1)], acc[m]);
                }
            }
#undef VD_T1READ
            if constexpr (!W1_STAT) {   // next tile's W1 (consumed after the next top-of-tile vmcnt(0))
#pragma unroll
                for (int s = 0; s < KS1; ++s)
                    w1f[s] = __builtin_amdgcn_raw_buffer_load_b128(rw1, lo16, (jn * KS1 + s) * 1024, 0);
            }
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                const float v0 = acc[m][0] * s2v.x + h2v.x, v1 = acc[m][1] * s2v.y + h2v.y;
                const float v2 = acc[m][2] * s2v.z + h2v.z, v3 = acc[m][3] * s2v.w + h2v.w;
                const t16x4_t o = {(E16)(v0 > 0.f ? v0 : 0.f), (E16)(v1 > 0.f ? v1 : 0.f),
                                   (E16)(v2 > 0.f ? v2 : 0.f), (E16)(v3 > 0.f ? v3 : 0.f)};
                *(t16x4_t*)(lt2 + lds_off(16 * (4 * half + m) + li, 2 * jn + (g >> 1)) + (g & 1) * 8) = o;
            }
        }
        VD_STAMP(4);
        // t2 complete. A plain s_barrier after this wave's LDS writes retire: the
        // fence of __syncthreads() would also wait for the next tile's x DMA
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        VD_STAMP(5);

        // ---- stage 3: out channels 32w..32w+31 (8 consecutive per lane), 8 tile rows ----
        {
            const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc(
                (void*)((E16*)a.y + (size_t)b * fpx * CO), 0, (int)(fpx * CO * 2), 0x00020000);
            const int ox = ox0 + li;
            const unsigned yo = ox < a.W ? (unsigned)((oy0 * a.W + ox) * CO + 32 * w + 8 * g) * 2u : 0x80000000u;
            // t2 (and, DS, x) fragments of row m+1 go out before the MFMAs of row m
            constexpr int NF = DS ? 2 + KS1 : 2;
            u32x4 fr[2][NF];
#define VD_T2READ(M, BUF)                                                                          \
            do {                                                                                   \
                _Pragma("unroll") for (int s_ = 0; s_ < 2; ++s_)                                   \
                    fr[BUF][s_] = *(const u32x4*)(lt2 + lds_off(16 * (M) + li, 4 * s_ + g));       \
                if constexpr (DS) {   /* downsample input: the tile's own pixels from LX */        \
                    const int r_ = ((M) + 1) * HWD + li + 1;                                       \
                    _Pragma("unroll") for (int s_ = 0; s_ < KS1; ++s_)                             \
                        fr[BUF][2 + (s_ < KS1 ? s_ : 0)] =                                         \
                            *(const u32x4*)(lxc + r_ * XROW + (lx_chunk<CIN>(r_, 4 * s_ + g) << 4)); \
                }                                                                                  \
            } while (0)
            VD_T2READ(0, 0);
#pragma unroll
            for (int m = 0; m < 8; ++m) {
                asm volatile("" ::: "memory");
                if (m + 1 < 8) VD_T2READ(m + 1, (m + 1) & 1);
                const u32x4* tf = fr[m & 1];
                const u32x4* xc = fr[m & 1] + 2;
                f32x4_t acc[2], accd[DS ? 2 : 1];
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    acc[j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                    for (int s = 0; s < 2; ++s) acc[j] = mfma(w3f[j][s], tf[s], acc[j]);
                    if constexpr (DS) {
                        accd[j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                        for (int s = 0; s < KS1; ++s) accd[j] = mfma(wdf[j][s], xc[s], accd[j]);
                    }
                }
                float v[8];
#pragma unroll
                for (int e = 0; e < 8; ++e) v[e] = acc[e >> 2][e & 3] * s3[e] + h3[e];
                if constexpr (DS) {   // + bn(downsample(x)), as the dual streaming kernel
#pragma unroll
                    for (int e = 0; e < 8; ++e) v[e] += accd[e >> 2][e & 3] * sd[e] + hd[e];
                } else {              // + identity
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        v[2 * e] += HT::lo(rf[m][e]);
                        v[2 * e + 1] += HT::hi(rf[m][e]);
                    }
                }
                typename HT::V8 o;
#pragma unroll
                for (int e = 0; e < 8; ++e) o[e] = (E16)(v[e] > 0.f ? v[e] : 0.f);
                // pixels past the frame: out-of-range lane offset, the store is dropped
                const unsigned so = oy0 + m < a.H ? yo + (unsigned)(m * a.W * CO * 2) : 0x80000000u;
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, o), ry, so, 0, 0);
            }
#undef VD_T2READ
        }
        if ((a.mode & 1) && t + tstep < tend) {   // experiment: no overlap of the x DMA
            __syncthreads();
            issue_x(t + tstep, DS ? buf ^ 1 : 0);
        }
        if constexpr (DS) buf ^= 1;
        VD_STAMP(6);
    }
    if (dg && lane == 0)
        for (int i = 0; i < 8; ++i) a.diag[i] = dsum[i];
#undef VD_STAMP
}

template <int CIN, bool DS, bool F16>
hipError_t launch(const BlockArgs& a, hipStream_t s) {
    constexpr int RPI = 1024 / (CIN * 2);
    constexpr size_t xb = (size_t)((HROWS + RPI - 1) / RPI * RPI) * CIN * 2;
    constexpr size_t lds = (DS ? 2 : 1) * xb + 192 * 128 + 128 * 128 + 1024;
    static const int cus = [] {
        (void)hipFuncSetAttribute((const void*)bottleneck_kernel<CIN, DS, F16>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        int dev = 0, n = 256;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
        return n > 0 ? n : 256;
    }();
    const int tiles = a.B * a.tiles_x * a.tiles_y;
    const int grid = tiles < cus ? tiles : cus;            // persistent: one workgroup per CU
    hipLaunchKernelGGL((bottleneck_kernel<CIN, DS, F16>), dim3(grid), dim3(512), lds, s, a);
    return hipGetLastError();
}

}  // namespace

bool vd_block_ok(int cin, bool ds, int h, int w) {
    if (!((cin == 256 && !ds) || (cin == 64 && ds))) return false;
    return h > 0 && w > 0 && (double)h * w * cin * 2 < 2147483647.0 && (double)h * w * CO * 2 < 2147483647.0;
}

hipError_t vd_launch_block(const BlockArgs& a, hipStream_t s) {
    if (a.B <= 0) return hipSuccess;
    if (a.cin == 256 && !a.ds) return a.f16 ? launch<256, false, true>(a, s) : launch<256, false, false>(a, s);
    if (a.cin == 64 && a.ds) return a.f16 ? launch<64, true, true>(a, s) : launch<64, true, false>(a, s);
    return hipErrorInvalidValue;
}
