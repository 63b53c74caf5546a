// conv_persist.hip — persistent form of the bf16 implicit-GEMM conv (conv.hip)
// for layers whose K loop is short (3x3 over 64 channels, 1x1 over 512: 8-18 K
// tiles). In the one-tile-per-workgroup kernel such a layer spends a large share of
// every tile on the prologue (two K tiles of DMA latency before the first MFMA) and
// the epilogue (LDS staging + stores, no loads in flight). Here a workgroup walks
// tiles, and the epilogue runs from registers (no LDS staging): the MFMAs compute
// D^T = W . X^T with the weight rows read in a pair permutation, so each lane ends
// with 8 consecutive output channels of one pixel -> BN / residual / activation in
// registers and one 16-B store per (M tile, channel pair). Both K buffers are then
// free as soon as the K loop ends, and the NEXT tile's first two K tiles are DMA'd
// before this tile's epilogue, which hides their latency; the residual and BN
// operands of a tile are loaded at its start. Same tile math and LDS image, same
// arithmetic (bf16 operands, f32 accumulate, acc*scale + shift, residual, activation)
// as conv_igemm_kernel<__bf16, BM, BN, 256, 2, true, true>.
//
// vmcnt bookkeeping (loads, stores and LDS-DMA retire in issue order). Per tile:
//   [K0, K1 (issued under the previous epilogue)] [previous tile's NST stores]
//   top: vmcnt(NST) -> K0, K1 landed
//   epilogue operands (NBN + NST loads), then K(kt+2) after the MFMAs of kt
//   kt = 1 waits vmcnt(NBN + NST [+ LPT]); kt >= 2 waits vmcnt(LPT or 0)
// Stores go through a buffer descriptor and are issued unconditionally (off-range
// offsets are dropped) so every thread issues exactly NST of them.
#include "vd_common.h"

#include <algorithm>
#include <cstdlib>

namespace {

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void_t;

__device__ __forceinline__ int lds_off(int row, int chunk) {
    return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4);
}

__device__ __forceinline__ float act_apply(float v, int act, float slope) {
    if (act == VD_ACT_RELU) return v > 0.f ? v : 0.f;
    if (act == VD_ACT_LEAKY) return v > 0.f ? v : v * slope;
    if (act == VD_ACT_SILU) return v / (1.0f + __expf(-v));
    return v;
}

template <int N>
__device__ __forceinline__ void wait_vm() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int BM, int BN>
__global__ __launch_bounds__(256) void conv_persist_kernel(ConvArgs a, int ntiles) {
    constexpr int NT = 256, VEC = 8, BKE = 64;
    constexpr int WAVES = 4;
    constexpr int WAVES_N = (BN >= 64 && BM < 4 * BN) ? 2 : 1;
    constexpr int WAVES_M = WAVES / WAVES_N;
    constexpr int WTM = BM / WAVES_M, WTN = BN / WAVES_N;
    constexpr int TM = WTM / 16, TN = WTN / 16;
    constexpr int NP = TN / 2;                            // 32-channel pairs of N tiles per wave
    constexpr int ROWS = NT / 8;
    constexpr int A_IT = BM / ROWS, B_IT = BN / ROWS;
    constexpr int LPT = A_IT + B_IT;                      // DMA instructions per lane per K tile
    constexpr int BUF = (BM + BN) * 128;
    constexpr int NST = TM * NP;                          // 16-B stores (and residual loads) per lane per tile
    constexpr int NBN = 4 * NP;                           // BN scale/shift loads (float4) per lane per tile
    static_assert(TN % 2 == 0, "pairs of 16-channel tiles");
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* kb0 = smem;                     // K tile kt lives in kb0 (kt even) / kb1 (kt odd)
    char* kb1 = smem + BUF;

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid / WAVES_N, wn = wid % WAVES_N;
    const int li = lane & 15, g = lane >> 4;
    const int chunk = tid & 7, rbase = tid >> 3;
    const int lchunk = chunk ^ ((rbase >> 1) & 7);
    const int nk = a.kpad / BKE;
    const int ohw = a.yh * a.yw;
    const long tap_dy = (long)a.xw * a.ldx;
    const long xbytes = (long)a.B * a.xh * a.xw * a.ldx * 2;
    const __amdgpu_buffer_rsrc_t rsrc_x =
        __builtin_amdgcn_make_buffer_rsrc((void*)a.x, 0, (int)(xbytes < 0x7fffffffL ? xbytes : 0x7fffffffL), 0x00020000);
    const __amdgpu_buffer_rsrc_t rsrc_w = __builtin_amdgcn_make_buffer_rsrc((void*)a.w, 0, 0x7fffffff, 0x00020000);
    const long ybytes = ((long)a.M - 1) * a.ldy * 2 + (long)(a.ycoff + a.cout) * 2;
    const __amdgpu_buffer_rsrc_t rsrc_y =
        __builtin_amdgcn_make_buffer_rsrc(a.y, 0, (int)(ybytes < 0x7fffffffL ? ybytes : 0x7fffffffL), 0x00020000);
    const __bf16* xsafe = (const __bf16*)a.x;

    // tiles of this workgroup: XCD-aware bijective start, then stride gridDim.x
    const int nwg = gridDim.x, bid = blockIdx.x;
    const int q8 = nwg >> 3, r8 = nwg & 7, xcd = bid & 7;
    const int first = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);

    // per-tile A-row state (input position of each of this thread's A rows at tap 0)
    long pix0[A_IT];
    int iy0[A_IT], ix0[A_IT];
    unsigned woff_g = 0;
    int t_kh = 0, t_kw = 0, t_c = 0;     // dense (kh, kw, c) tracker of the next K tile to issue
    auto setup = [&](int t) {
        const int tn = t % a.ntiles_n, tm = t / a.ntiles_n;
        const int m0 = tm * BM, n0 = tn * BN;
#pragma unroll
        for (int i = 0; i < A_IT; ++i) {
            const int m = m0 + rbase + ROWS * i;
            if (m < a.M) {
                const int b = m / ohw, rem = m - b * ohw;
                const int oy = rem / a.yw, ox = rem - oy * a.yw;
                iy0[i] = oy * a.stride - a.pad;
                ix0[i] = ox * a.stride - a.pad;
                pix0[i] = (((long)b * a.xh + iy0[i]) * a.xw + ix0[i]) * a.ldx + a.xcoff;
            } else {
                iy0[i] = -(1 << 28); ix0[i] = 0; pix0[i] = 0;
            }
        }
        woff_g = (unsigned)(((long)(n0 + rbase) * a.kpad + lchunk * VEC) * 2);
        t_kh = t_kw = t_c = 0;
    };
    // next K tile (tracker order) of the current A-row state into `buf` (lane-linear
    // DMA, swizzle on the source; padding taps read zeros past num_records)
    auto issue = [&](int kt, char* buf) {
        const int dy = t_kh, dx = t_kw, c = t_c + lchunk * VEC;
        char* As_ = buf;
        char* Bs_ = As_ + BM * 128;
        const long toff = dy * tap_dy + (long)dx * a.ldx + c;
#pragma unroll
        for (int i = 0; i < A_IT; ++i) {
            const int iy = iy0[i] + dy, ix = ix0[i] + dx;
            const bool ok = (unsigned)iy < (unsigned)a.xh && (unsigned)ix < (unsigned)a.xw;
            const unsigned off = ok ? (unsigned)((pix0[i] + toff) * 2) : 0x80000000u;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc_x, (lds_void_t*)(As_ + (wid * 8 + ROWS * i) * 128), 16, off,
                                                     0, 0, 0);
        }
#pragma unroll
        for (int i = 0; i < B_IT; ++i)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc_w, (lds_void_t*)(Bs_ + (wid * 8 + ROWS * i) * 128), 16,
                                                     woff_g + (unsigned)(ROWS * i * a.kpad * 2),
                                                     (unsigned)(kt * BKE * 2), 0, 0);
        t_c += BKE;
        if (t_c >= a.cin_pad) { t_c = 0; if (++t_kw == a.kw) { t_kw = 0; ++t_kh; } }
    };

    int t = first;
    if (t >= ntiles) return;
    setup(t);
    issue(0, kb0);
    if (nk > 1) issue(1, kb1);
#pragma unroll 1
    for (; t < ntiles; t += nwg) {
        const int tn_ = t % a.ntiles_n, tm_ = t / a.ntiles_n;
        const int m0 = tm_ * BM, n0 = tn_ * BN;
        // K0 / K1 of this tile: the previous tile's NST stores are the only younger ops
        // and may fly on; before the first tile nothing follows them
        if (t == first) wait_vm<0>(); else wait_vm<NST>();
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");

        // epilogue operands of this tile, loaded now (after the K-loop DMAs they would
        // retire only behind them): lane (li, g) of wave column wn owns, per M tile i and
        // channel pair p, pixel m0 + wm*WTM + 16i + li and channels c(p) .. +8 with
        // c(p) = n0 + wn*WTN + 32p + 8g (weight rows read permuted below)
        u32x4 rpf[TM][NP];
        float4 scv[NP][2], shv[NP][2];
        const bool pf = a.res_mode != VD_RES_NONE;
#pragma unroll
        for (int p = 0; p < NP; ++p) {
            const int c = n0 + wn * WTN + 32 * p + 8 * g;
            const int cc = c < a.cout ? c : 0;
            scv[p][0] = *(const float4*)(a.scale + cc);
            scv[p][1] = *(const float4*)(a.scale + cc + 4);
            shv[p][0] = *(const float4*)(a.shift + cc);
            shv[p][1] = *(const float4*)(a.shift + cc + 4);
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                const int m = m0 + wm * WTM + 16 * i + li;
                const bool ok = pf && m < a.M && c < a.cout;
                size_t roff = 0;
                if (ok) {
                    if (a.res_up) {
                        const int b = m / ohw, rem = m - b * ohw;
                        const int oy = rem / a.yw, ox = rem - oy * a.yw;
                        roff = ((size_t)(b * a.rh + (oy >> 1)) * a.rw + (ox >> 1)) * a.res_ld + a.res_coff + c;
                    } else {
                        roff = (size_t)m * a.res_ld + a.res_coff + c;
                    }
                }
                rpf[i][p] = *(const u32x4*)(ok ? (const __bf16*)a.res + roff : xsafe);
            }
        }

        f32x4_t acc[TM][TN];
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
        // D^T = W . X^T: A operand = weight rows (B tile), read in the pair permutation
        // (tile j, MFMA row r -> channel 32(j>>1) + 8(r>>2) + 4(j&1) + (r&3)), so a lane
        // ends with 8 consecutive channels of one pixel per pair of tiles
        const int prow = 8 * (li >> 2) + (li & 3);
        auto step = [&](int kt, char* buf) {
            if (kt == 1) {
                if (nk > 2) wait_vm<NST + NBN + LPT>(); else wait_vm<NST + NBN>();
            } else if (kt >= 2) {
                if (kt + 1 < nk) wait_vm<LPT>(); else wait_vm<0>();
            }
            if (kt > 0) __builtin_amdgcn_s_barrier();
            const char* As = buf;
            const char* Bs = As + BM * 128;
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) {
                const int ch = ks * 4 + g;
                u32x4 af[TM], bfr[TN];
#pragma unroll
                for (int i = 0; i < TM; ++i) af[i] = *(const u32x4*)(As + lds_off(wm * WTM + i * 16 + li, ch));
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    bfr[j] = *(const u32x4*)(Bs + lds_off(wn * WTN + 32 * (j >> 1) + 4 * (j & 1) + prow, ch));
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, bfr[j]),
                                                                           __builtin_bit_cast(bf16x8_t, af[i]),
                                                                           acc[i][j], 0, 0, 0);
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            if (kt + 2 < nk) issue(kt + 2, buf);
        };
        // unrolled by two: the buffer of every K tile is a compile-time choice
        for (int kt = 0; kt < nk; kt += 2) {
            step(kt, kb0);
            if (kt + 1 < nk) step(kt + 1, kb1);
        }
        // epilogue operands landed (a builtin wait the compiler sees: no wait of its own,
        // which would also cover the DMAs below, lands in the epilogue); then both K
        // buffers are free and the next tile's first two K tiles go out under the epilogue
        __builtin_amdgcn_s_waitcnt(0x0F70);
        if (t + nwg < ntiles) {
            setup(t + nwg);
            issue(0, kb0);
            if (nk > 1) issue(1, kb1);
        }
        asm volatile("" ::: "memory");

        // ---- register epilogue: BN, residual, activation, 16-B stores ----
        const bool pre = a.res_mode == VD_RES_PRE_ACT, post = a.res_mode == VD_RES_POST_ACT;
        const bool relu = a.act == VD_ACT_RELU, leaky = a.act == VD_ACT_LEAKY, silu = a.act == VD_ACT_SILU;
#pragma unroll
        for (int i = 0; i < TM; ++i) {
            const int m = m0 + wm * WTM + 16 * i + li;
#pragma unroll
            for (int p = 0; p < NP; ++p) {
                const int c = n0 + wn * WTN + 32 * p + 8 * g;
                const float sc[8] = {scv[p][0].x, scv[p][0].y, scv[p][0].z, scv[p][0].w,
                                     scv[p][1].x, scv[p][1].y, scv[p][1].z, scv[p][1].w};
                const float sh[8] = {shv[p][0].x, shv[p][0].y, shv[p][0].z, shv[p][0].w,
                                     shv[p][1].x, shv[p][1].y, shv[p][1].z, shv[p][1].w};
                const bf16x8_t rb8 = __builtin_bit_cast(bf16x8_t, rpf[i][p]);
                float v[8];
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    v[e] = acc[i][2 * p + (e >> 2)][e & 3] * sc[e] + sh[e];
                    v[e] = pre ? v[e] + (float)rb8[e] : v[e];
                }
                if (silu) {
#pragma unroll
                    for (int e = 0; e < 8; ++e) v[e] = act_apply(v[e], VD_ACT_SILU, 0.f);
                } else {
#pragma unroll
                    for (int e = 0; e < 8; ++e) {
                        const float r = v[e] > 0.f ? v[e] : 0.f;
                        const float l = v[e] > 0.f ? v[e] : v[e] * a.slope;
                        v[e] = relu ? r : (leaky ? l : v[e]);
                    }
                }
                bf16x8_t o;
#pragma unroll
                for (int e = 0; e < 8; ++e) o[e] = (__bf16)(post ? v[e] + (float)rb8[e] : v[e]);
                const bool ok = m < a.M && c < a.cout;
                const unsigned off = ok ? (unsigned)((((long)m * a.ldy + a.ycoff + c)) * 2) : 0x80000000u;
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, o), rsrc_y, off, 0, 0);
            }
        }
    }
}

template <int BM, int BN>
hipError_t launch(const ConvArgs& a0, hipStream_t s) {
    ConvArgs a = a0;
    a.ntiles_n = (a.cout + BN - 1) / BN;
    const int ntiles = ((a.M + BM - 1) / BM) * a.ntiles_n;
    constexpr size_t lds = 2 * (size_t)(BM + BN) * 128;
    static const int cus = [] {
        (void)hipFuncSetAttribute((const void*)conv_persist_kernel<BM, BN>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)lds);
        int dev = 0, n = 256;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
        return n > 0 ? n : 256;
    }();
    const int per_cu = (int)(160 * 1024 / lds) < 2 ? 1 : (int)std::min<size_t>(4, 160 * 1024 / lds);
    const int grid = std::min(ntiles, per_cu * cus);
    hipLaunchKernelGGL((conv_persist_kernel<BM, BN>), dim3(grid), dim3(256), lds, s, a, ntiles);
    return hipGetLastError();
}

}  // namespace

// bf16, dense taps (Cin a multiple of 64), 16-B aligned output/residual slices, bf16
// output; VD_CONV_PERSIST: max K tiles (0 = off). OFF by default: measured
// (tools/convbench, B=64) level with the one-shot GEMM on the N=64 layers (-4..+6 %)
// and behind it on N=128 (m=61440: 23 -> 36 us; 409600x128x512: 145 -> 180 us) --
// the static tile split leaves up to one tile per workgroup of imbalance in the
// last round, more than the hidden prologue/epilogue saves.
bool vd_conv_persist_ok(const ConvArgs& a) {
    const char* e = getenv("VD_CONV_PERSIST");
    const int kmax = e ? atoi(e) : 0;
    if (kmax <= 0 || a.out_f32 || a.x2) return false;
    if ((a.cin_pad % 64) != 0 || a.kpad / 64 > kmax || a.kpad / 64 < 1) return false;
    if ((a.cout & 7) || (a.ldy & 7) || (a.ycoff & 7) || ((a.ldx | a.xcoff) & 7)) return false;
    if (a.res_mode != VD_RES_NONE && ((a.res_ld | a.res_coff) & 7)) return false;
    if ((long)a.M * a.ldy * 2 >= 0x7fffffffL) return false;
    return true;
}

hipError_t vd_launch_conv_persist(const ConvArgs& a, hipStream_t s) {
    const int bn = a.cout <= 32 ? 32 : (a.cout <= 64 ? 64 : 128);
    const long tiles128 = (long)((a.M + 127) / 128) * ((a.cout + bn - 1) / bn);
    const char* e = getenv("VD_CONV_PERSIST_SMALL");   // tests force either row tile
    const long small_lim = e ? atol(e) : 512;
    if (tiles128 < small_lim) {   // small grids: 64-row tiles (as the one-shot kernel)
        if (bn == 32) return launch<64, 32>(a, s);
        if (bn == 64) return launch<64, 64>(a, s);
        return launch<64, 128>(a, s);
    }
    if (bn == 32) return launch<128, 32>(a, s);
    if (bn == 64) return launch<128, 64>(a, s);
    return launch<128, 128>(a, s);
}
