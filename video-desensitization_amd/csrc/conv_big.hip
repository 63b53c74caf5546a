// conv_big.hip — 256 x 256-tile implicit-GEMM convolution for the large dense
// bf16 layers (Cout a multiple of 256, Cin a multiple of 64): ResNet layer3/4
// 3x3 and 1x1 convs, FPN lateral/merge convs.
//
// Same arithmetic contract as conv.hip (bf16 operands, f32 MFMA accumulation,
// fused BN scale/shift + residual + activation, K order (kh, kw, c)); different
// schedule, built so the K pipeline never drains at a barrier:
//   * 8 waves; each wave owns a 64 x 32 block in each of the four 128 x 128
//     quadrants of the 256 x 256 tile (`acc` below), so one quadrant is computed
//     per PHASE from one A half-tile and one B half-tile.
//   * A K tile (64 deep, 128-B rows) is four 16-KB half-tiles A0 (rows 0-127),
//     B0 (channels 0-127), B1, A1, staged by LDS-DMA (global_load_lds_dwordx4,
//     source-side XOR swizzle) into two K stages (128 KB of LDS, 1 workgroup/CU).
//   * Phases run (A0,B0) (A0,B1) (A1,B1) (A1,B0): A fragments are read once per
//     half, B0 is kept in registers across the K tile. Two raw barriers per
//     phase; waves 4-7 run one barrier behind waves 0-3, so on every SIMD one
//     wave issues its fragment reads and DMA while the other multiplies.
//     Half-tile h is issued 6 phases before its first use and retired by a
//     counted s_waitcnt vmcnt (never 0 in steady state); a slot is refilled only
//     two phases after its last read (the skew rule; proof in DESIGN.md).
//   * Epilogue: the f32 tile goes through LDS 64 rows at a time, 16-B stores.
#include "vd_common.h"
#include <algorithm>

namespace {

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void_t;

__device__ __attribute__((aligned(16))) unsigned vdb_zero16[4] = {0u, 0u, 0u, 0u};

#ifdef VD_STAMPS   // diagnostic build only (tools/stamps.cpp): s_memtime at segment edges
__device__ unsigned long long vd_stamps[8][2048];
#define VDB_STAMP()                                                                            \
    do {                                                                                       \
        if (blockIdx.x == 0 && lane == 0 && sidx < 2048) vd_stamps[wid][sidx++] = __builtin_amdgcn_s_memtime(); \
    } while (0)
#else
#define VDB_STAMP() do { } while (0)
#endif
#ifndef VDB_DIAG_DMA          // diagnostic builds (tools/stamps.cpp) may drop the DMA or the
#define VDB_DIAG_DMA 1        // fragment reads to price them; results are then meaningless
#endif
#ifndef VDB_DIAG_READ
#define VDB_DIAG_READ 1
#endif

constexpr int HT = 16384;          // half-tile bytes: 128 rows x 128 B
constexpr int LDS_BYTES = 8 * HT;  // 2 stages x {A0, B0, B1, A1}
constexpr int EPLD = 256 + 4;      // f32 epilogue row stride

__device__ __forceinline__ int lds_off(int row, int chunk) {
    return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4);
}

__device__ __forceinline__ float act_apply(float v, int act, float slope) {
    if (act == VD_ACT_RELU) return v > 0.f ? v : 0.f;
    if (act == VD_ACT_LEAKY) return v > 0.f ? v : v * slope;
    if (act == VD_ACT_SILU) return v / (1.0f + __expf(-v));
    return v;
}

// s_waitcnt vmcnt(2*n) for a runtime n in [0, 4]
__device__ __forceinline__ void wait_halves(int n) {
    switch (n) {
        case 0: asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory"); break;
        case 1: asm volatile("s_waitcnt vmcnt(2) lgkmcnt(0)" ::: "memory"); break;
        case 2: asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)" ::: "memory"); break;
        case 3: asm volatile("s_waitcnt vmcnt(6) lgkmcnt(0)" ::: "memory"); break;
        default: asm volatile("s_waitcnt vmcnt(8) lgkmcnt(0)" ::: "memory"); break;
    }
}

// s_waitcnt vmcnt(2*n) only (LDS reads stay in flight)
__device__ __forceinline__ void wait_vm(int n) {
    switch (n) {
        case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
        case 1: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
        case 2: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
        case 3: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
        default: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    }
}

// F16: the fp16 plan (VD_PREC_FP16) on fp16 operands / activations, else bf16
template <bool F16>
__global__ __launch_bounds__(512) void conv_big_kernel(ConvArgs a) {
    using H16 = Half16<F16>;
    typedef typename H16::T T;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wr = wid >> 2, wc = wid & 3;            // wave row (0..1) / column (0..3)

    // XCD-aware bijective remap: blocks sharing an XCD take consecutive tiles
    const int nwg = gridDim.x, bid = blockIdx.x;
    const int q8 = nwg >> 3, r8 = nwg & 7, xcd = bid & 7;
    const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
    const int tn = wg % a.ntiles_n, tm = wg / a.ntiles_n;
    const int m0 = tm * 256, n0 = tn * 256;

    // DMA roles: lane loads 16-B chunk `lchunk` of tile rows rbase + 64*i
    const int rbase = tid >> 3;
    const int lchunk = (tid & 7) ^ ((rbase >> 1) & 7);
    const int ohw = a.yh * a.yw;
    // Per A row: the pixel's input position at tap (0,0) and its element offset
    // there (may point before the image; used only when the tap is inside).
    int iy0[4], ix0[4];
    long pix0[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int m = m0 + rbase + 64 * i;
        if (m < a.M) {
            const int b = m / ohw, rem = m - b * ohw;
            const int oy = rem / a.yw, ox = rem - oy * a.yw;
            iy0[i] = oy * a.stride - a.pad;
            ix0[i] = ox * a.stride - a.pad;
            pix0[i] = (((long)b * a.xh + iy0[i]) * a.xw + ix0[i]) * a.ldx + a.xcoff + lchunk * 8;
        } else {
            iy0[i] = -(1 << 28); ix0[i] = 0; pix0[i] = 0;
        }
    }
    // A K tiles are issued in order (A0 of tile t before A0 of t+1, likewise A1):
    // two incremental (dy, dx, c) trackers replace per-issue divisions. The
    // element offset of tap (dy, dx), channel c relative to tap (0,0) is uniform.
    int a0_dy = 0, a0_dx = 0, a0_c = 0, a1_dy = 0, a1_dx = 0, a1_c = 0;
    const long tap_dy = (long)a.xw * a.ldx;
    const int nk = a.kpad / 64;
    const int nh_total = 4 * nk;                      // half-tiles in the K loop
    // LDS-DMA through buffer descriptors (buffer_load_dwordx4 ... lds): 32-bit per-lane
    // byte offsets, and out-of-range offsets return zeros (conv padding). Built from
    // kernel arguments only, so the descriptors are scalar.
    const __amdgpu_buffer_rsrc_t rsrc_x = __builtin_amdgcn_make_buffer_rsrc(
        (void*)a.x, 0, (int)((long)a.B * a.xh * a.xw * a.ldx * 2 < 0x7fffffffL ? (long)a.B * a.xh * a.xw * a.ldx * 2
                                                                                 : 0x7fffffffL), 0x00020000);
    const __amdgpu_buffer_rsrc_t rsrc_w = __builtin_amdgcn_make_buffer_rsrc((void*)a.w, 0, 0x7fffffff, 0x00020000);
    const unsigned woff = (unsigned)(((long)(n0 + rbase) * a.kpad + lchunk * 8) * 2);

    // Issue half-tile h (K tile h>>2, part h&3 in {A0, B0, B1, A1}) into its slot.
#define VDB_ISSUE(h_)                                                                          \
    do {                                                                                       \
        const int hh = (h_);                                                                   \
        const int t_ = hh >> 2, j_ = hh & 3;                                                   \
        char* dst_ = smem + ((t_ & 1) * 4 + j_) * HT + wid * 8 * 128;                          \
        const int kpos = t_ * 64;                                                              \
        if (j_ == 0 || j_ == 3) {                                                              \
            int& dy = j_ == 3 ? a1_dy : a0_dy;                                                 \
            int& dx = j_ == 3 ? a1_dx : a0_dx;                                                 \
            int& cc = j_ == 3 ? a1_c : a0_c;                                                   \
            const long toff = dy * tap_dy + (long)dx * a.ldx + cc;                             \
            const int i0 = j_ == 3 ? 2 : 0;                                                    \
            _Pragma("unroll") for (int ii = 0; ii < 2; ++ii) {                                 \
                const int i = i0 + ii;                                                         \
                const bool ok = (unsigned)(iy0[i] + dy) < (unsigned)a.xh &&                   \
                                (unsigned)(ix0[i] + dx) < (unsigned)a.xw;                      \
                /* padding taps: an offset past num_records, which the buffer unit reads as 0 */ \
                const unsigned off = ok ? (unsigned)((pix0[i] + toff) * 2) : 0x80000000u;      \
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc_x, (lds_void_t*)(dst_ + ii * 64 * 128), 16, \
                                                         off, 0, 0, 0);                        \
            }                                                                                  \
            cc += 64;                                                                          \
            if (cc >= a.cin_pad) { cc = 0; if (++dx == a.kw) { dx = 0; ++dy; } }              \
        } else {                                                                               \
            const int i0 = j_ == 2 ? 2 : 0;                                                    \
            _Pragma("unroll") for (int ii = 0; ii < 2; ++ii)                                   \
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc_w, (lds_void_t*)(dst_ + ii * 64 * 128), 16, \
                                                         woff + (unsigned)(64 * (i0 + ii) * a.kpad * 2), \
                                                         (unsigned)(kpos * 2), 0, 0);          \
        }                                                                                      \
    } while (0)

    // acc[mh][nh][i][jn]: rows mh*128 + wr*64 + i*16 (+frag), cols nh*128 + wc*32 + jn*16
    f32x4_t acc[2][2][4][2];
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y)
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) acc[x][y][i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    u32x4 af[4][2], b0[2][2], b1[2][2];

    // Staggered schedule: two barriers per phase, L_p = {fragment reads of
    // phase p, refill of half-tile p+6, vmcnt for what phase p+1 reads} | X_p |
    // C_p = {16 MFMAs} | Y_p. Waves 4-7 run one barrier behind waves 0-3, so on
    // every SIMD (waves s and s+4) one wave loads while the other multiplies.
    // B0 stays in registers from phase 0 to phase 3, so a slot's last read is in
    // phase 4t (A0, B0), 4t+1 (B1) or 4t+2 (A1); with the one-barrier skew a
    // refill must come >= 2 phases after the last read: run-ahead 6.
#define VDB_SPHASE(R, MH, NH, RA, RB0, RB1, STEADY)                                            \
    do {                                                                                       \
        const int p = 4 * t + (R);                                                             \
        const char* st_ = smem + (t & 1) * 4 * HT;                                             \
        VDB_STAMP();                                                                           \
        /* DMA issue first: its cost overlaps the fragment reads' latency */                  \
        if (VDB_DIAG_DMA && p + 6 < nh_total) VDB_ISSUE(p + 6);                                \
        if ((RA) && VDB_DIAG_READ) {                                                           \
            const char* As_ = st_ + ((MH) ? 3 : 0) * HT;                                       \
            _Pragma("unroll") for (int i = 0; i < 4; ++i)                                      \
            _Pragma("unroll") for (int ks = 0; ks < 2; ++ks)                                   \
                af[i][ks] = *(const u32x4*)(As_ + lds_off(wr * 64 + i * 16 + (lane & 15), ks * 4 + (lane >> 4))); \
        }                                                                                      \
        if ((RB0) && VDB_DIAG_READ) {                                                          \
            _Pragma("unroll") for (int j = 0; j < 2; ++j)                                      \
            _Pragma("unroll") for (int ks = 0; ks < 2; ++ks)                                   \
                b0[j][ks] = *(const u32x4*)(st_ + HT + lds_off(wc * 32 + j * 16 + (lane & 15), ks * 4 + (lane >> 4))); \
        }                                                                                      \
        if ((RB1) && VDB_DIAG_READ) {                                                          \
            _Pragma("unroll") for (int j = 0; j < 2; ++j)                                      \
            _Pragma("unroll") for (int ks = 0; ks < 2; ++ks)                                   \
                b1[j][ks] = *(const u32x4*)(st_ + 2 * HT + lds_off(wc * 32 + j * 16 + (lane & 15), ks * 4 + (lane >> 4))); \
        }                                                                                      \
        VDB_STAMP();                                                                           \
        if (STEADY) {                                                                          \
            if ((R) == 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");                     \
            else asm volatile("s_waitcnt vmcnt(6)" ::: "memory");                              \
        } else if (p + 1 < nh_total) {                                                         \
            const int q = p + 1;                                                               \
            const int need = 4 * (q >> 2) + ((q & 3) == 0 ? 1 : ((q & 3) == 1 ? 2 : 3));       \
            wait_vm(min(p + 5, nh_total - 1) - need);                                          \
        }                                                                                      \
        VDB_STAMP();                                                                           \
        __builtin_amdgcn_s_barrier();                                                          \
        VDB_STAMP();                                                                           \
        /* no lgkmcnt(0) here: hipcc waits per MFMA operand, and every read of this */         \
        /* phase is consumed (so complete) before the second barrier */                       \
        __builtin_amdgcn_s_setprio(1);                                                         \
        _Pragma("unroll") for (int ks = 0; ks < 2; ++ks)                                       \
        _Pragma("unroll") for (int i = 0; i < 4; ++i)                                          \
        _Pragma("unroll") for (int j = 0; j < 2; ++j)                                          \
            acc[MH][NH][i][j] = H16::mfma(af[i][ks], (NH) ? b1[j][ks] : b0[j][ks], acc[MH][NH][i][j]); \
        __builtin_amdgcn_s_setprio(0);                                                         \
        asm volatile("" ::: "memory");                                                         \
        VDB_STAMP();                                                                           \
        __builtin_amdgcn_s_barrier();                                                          \
        asm volatile("" ::: "memory");                                                         \
    } while (0)

    int t = 0;
#ifdef VD_STAMPS
    int sidx = 0;
#endif
    {
        for (int h = 0; h < 6 && h < nh_total; ++h) VDB_ISSUE(h);   // prologue: half-tiles 0..5
        wait_vm(min(5, nh_total - 1) - 1);                          // A0(0), B0(0) landed
        __builtin_amdgcn_s_barrier();
        if (wr == 1) __builtin_amdgcn_s_barrier();                  // the skew
        asm volatile("" ::: "memory");
        for (; t + 3 <= nk; ++t) {
            VDB_SPHASE(0, 0, 0, true, true, false, true);
            VDB_SPHASE(1, 0, 1, false, false, true, true);
            VDB_SPHASE(2, 1, 1, true, false, false, true);
            VDB_SPHASE(3, 1, 0, false, false, false, true);
        }
        for (; t < nk; ++t) {
            VDB_SPHASE(0, 0, 0, true, true, false, false);
            VDB_SPHASE(1, 0, 1, false, false, true, false);
            VDB_SPHASE(2, 1, 1, true, false, false, false);
            VDB_SPHASE(3, 1, 0, false, false, false, false);
        }
        if (wr == 0) __builtin_amdgcn_s_barrier();                  // undo the skew
    }
#undef VDB_SPHASE
#undef VDB_ISSUE
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();

    // ---- fused epilogue: 4 passes of 64 tile rows (pass p = quadrant row p>>1, wave row p&1) ----
    float* ep = (float*)smem;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        if (p) __syncthreads();
        if (wr == (p & 1)) {
#pragma unroll
            for (int nh = 0; nh < 2; ++nh)
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int j = 0; j < 2; ++j)
#pragma unroll
                        for (int r = 0; r < 4; ++r)
                            ep[(i * 16 + (lane >> 4) * 4 + r) * EPLD + nh * 128 + wc * 32 + j * 16 + (lane & 15)] =
                                acc[p >> 1][nh][i][j][r];
        }
        __syncthreads();
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
            const int it = tid + 512 * qq;
            const int row = it >> 5, cg = it & 31;
            const int m = m0 + (p >> 1) * 128 + (p & 1) * 64 + row;
            const int nb = n0 + cg * 8;
            if (m >= a.M) continue;
            const float* er = ep + row * EPLD + cg * 8;
            const float4 e0 = *(const float4*)er, e1 = *(const float4*)(er + 4);
            const float4 s0 = *(const float4*)(a.scale + nb), s1 = *(const float4*)(a.scale + nb + 4);
            const float4 h0 = *(const float4*)(a.shift + nb), h1 = *(const float4*)(a.shift + nb + 4);
            float v[8] = {e0.x * s0.x + h0.x, e0.y * s0.y + h0.y, e0.z * s0.z + h0.z, e0.w * s0.w + h0.w,
                          e1.x * s1.x + h1.x, e1.y * s1.y + h1.y, e1.z * s1.z + h1.z, e1.w * s1.w + h1.w};
            float rv[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
            if (a.res_mode != VD_RES_NONE) {
                size_t roff;
                if (a.res_up) {
                    const int b = m / ohw, rem = m - b * ohw;
                    const int oy = rem / a.yw, ox = rem - oy * a.yw;
                    roff = ((size_t)(b * a.rh + (oy >> 1)) * a.rw + (ox >> 1)) * a.res_ld + a.res_coff + nb;
                } else {
                    roff = (size_t)m * a.res_ld + a.res_coff + nb;
                }
                const typename H16::V8 r8 = *(const typename H16::V8*)((const T*)a.res + roff);
#pragma unroll
                for (int e = 0; e < 8; ++e) rv[e] = (float)r8[e];
            }
            typename H16::V8 o;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                float t = v[e];
                if (a.res_mode == VD_RES_PRE_ACT) t += rv[e];
                t = act_apply(t, a.act, a.slope);
                if (a.res_mode == VD_RES_POST_ACT) t += rv[e];
                o[e] = (T)t;
            }
            *(typename H16::V8*)((T*)a.y + (size_t)m * a.ldy + a.ycoff + nb) = o;
        }
    }
}


}  // namespace

// Eligible: bf16 dense taps (Cin a multiple of 64), Cout a multiple of 256, bf16
// output with 16-B aligned channel offsets, at least tune.conv_big 256 x 256 tiles.
// Measured (tools/convbench): at K = 512 ahead of the 128x128 GEMM by 14 % on the
// 409600 x 256 layers (layer3.0 conv1, FPN output1), level on the 25600 x 2048 ones.
bool vd_conv_big_ok(const ConvArgs& a) {
    const int min_tiles = a.tune->conv_big;
    if (min_tiles <= 0 || a.out_f32) return false;
    if ((a.cin_pad % 64) != 0 || (a.cout % 256) != 0 || a.kpad / 64 < 2 || a.kpad < a.tune->conv_big_kmin) return false;
    if (((a.ldy | a.ycoff) & 7) || ((a.ldx | a.xcoff) & 7)) return false;
    if (a.res_mode != VD_RES_NONE && ((a.res_ld | a.res_coff) & 7)) return false;
    const long tiles = (long)((a.M + 255) / 256) * (a.cout / 256);
    return tiles >= min_tiles;
}

hipError_t vd_launch_conv_big(const ConvArgs& a0, hipStream_t s) {
    static const bool attr = [] {
        (void)hipFuncSetAttribute((const void*)conv_big_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
        (void)hipFuncSetAttribute((const void*)conv_big_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
        return true;
    }();
    (void)attr;
    ConvArgs a = a0;
    a.ntiles_n = a.cout / 256;
    dim3 grid(((a.M + 255) / 256) * a.ntiles_n), block(512);
    if (a.f16) hipLaunchKernelGGL(conv_big_kernel<true>, grid, block, LDS_BYTES, s, a);
    else hipLaunchKernelGGL(conv_big_kernel<false>, grid, block, LDS_BYTES, s, a);
    return hipGetLastError();
}
