// conv.hip — NHWC implicit-GEMM convolution on CDNA4 MFMA.
//
// Replaces every nn.Conv2d + BatchNorm2d(eval) + activation of the RetinaFace
// forward (detect_face/retinaface.py:71-92 via torchvision resnet50 [ext],
// detect_face/nets/layers.py:10-66,79-114) and of the YOLOv8n plate forward.
//
//   GEMM view: D[m][n] = sum_k A[m][k] * B[n][k]
//     m = output pixel (b, oy, ox)                 M = B*OH*OW
//     n = output channel                           N = Cout
//     k = (kh, kw, c) with c fastest               K = KH*KW*Cin_pad
//   A is gathered from the NHWC input on the fly (zero outside the image =
//   conv padding); B is the weight packed [Npad][Kpad] at load time.
//
//   Block tile BM x BN x (128 bytes of K), 256 threads = 4 wave64s, each wave
//   a (BM/WAVES_M) x (BN/WAVES_N) sub-tile of 16x16 MFMA tiles. K tiles arrive
//   by LDS-DMA (buffer_load ... lds) in a double-buffered LDS image with 128-byte
//   rows and a (row>>1)&7 XOR swizzle on 16-byte chunks, which makes the
//   ds_read_b128 fragment reads of a 16x16x32 operand conflict-free.
//   bf16 mode : v_mfma_f32_16x16x32_bf16, one 16-B fragment per lane per step.
//   f32  mode : v_mfma_f32_16x16x4_f32 (exact f32), four MFMAs per 16-B fragment.
//   Epilogue (fused): y = acc*scale + shift (BN eval, same form as torch's
//   CPU inference kernel), optional residual add before/after the activation
//   (ResNet bottleneck; FPN lateral + nearest-2x upsample, layers.py:102-110),
//   activation (ReLU / LeakyReLU / SiLU), store at a channel offset.
//   Block -> tile mapping is XCD-aware: blocks that share an A (pixel) panel
//   are placed on one XCD so the panel is fetched into that XCD's L2 once.
#include "vd_common.h"
#include <algorithm>
#include <type_traits>

namespace {

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));   // native vector (HIP's uint4 is a struct)

template <typename T> struct Elem;
template <> struct Elem<__bf16> { static constexpr int VEC = 8; };
template <> struct Elem<_Float16> { static constexpr int VEC = 8; };
template <> struct Elem<float>  { static constexpr int VEC = 4; };

__device__ __forceinline__ int lds_off(int row, int chunk) {
    return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4);
}

__device__ __forceinline__ float act_apply(float v, int act, float slope) {
    if (act == VD_ACT_RELU) return v > 0.f ? v : 0.f;
    if (act == VD_ACT_LEAKY) return v > 0.f ? v : v * slope;
    if (act == VD_ACT_SILU) return v / (1.0f + __expf(-v));
    return v;
}

template <typename T>
__device__ __forceinline__ float load_elem(const void* p, size_t off) {
    if constexpr (std::is_same<T, float>::value) return ((const float*)p)[off];
    else return (float)((const T*)p)[off];
}

// 16 zero bytes: the LDS-DMA source of padding taps (conv zero padding, K padding).
__device__ __attribute__((aligned(16))) unsigned vd_zero16[4] = {0u, 0u, 0u, 0u};

typedef __attribute__((address_space(3))) void lds_void_t;

// NT threads (4 waves); two LDS stages: one K tile in flight, two barriers per K tile.
template <typename T, int BM, int BN, int NT, int STAGES, bool DENSE>
__global__ __launch_bounds__(NT) void conv_igemm_kernel(ConvArgs a) {
    constexpr int VEC = Elem<T>::VEC;
    constexpr int BKE = 8 * VEC;                 // K elements per 128-byte tile row
    constexpr int WAVES = NT / 64;
    // tall tiles (BM >= 4*BN) stack the waves along M: 64x64 wave tiles for BN = 64
    constexpr int WAVES_N = (BN >= 64 && BM < 4 * BN) ? 2 : 1;
    constexpr int WAVES_M = WAVES / WAVES_N;
    constexpr int WTM = BM / WAVES_M, WTN = BN / WAVES_N;
    constexpr int TM = WTM / 16, TN = WTN / 16;
    constexpr int ROWS = NT / 8;                 // tile rows covered by one pass of 16-B chunks
    constexpr int A_IT = BM / ROWS, B_IT = BN / ROWS;
    static_assert(BM % ROWS == 0 && BN % ROWS == 0 && STAGES == 2, "tile shape");
    constexpr int KSTEP = std::is_same<T, float>::value ? 16 : 32;  // K per fragment step
    constexpr int NKS = BKE / KSTEP;                                 // = 2
    constexpr int BUF = (BM + BN) * 128;
    constexpr int EPLD = BN + 4;                 // f32 epilogue row stride (conflict-free fragment writes)
    constexpr int CG = BN / 8;                   // 8-channel groups per output row
    constexpr int ITEMS = BM * CG / NT;          // epilogue items (row, 8 channels) per thread
    constexpr int EP = (ITEMS % 4 == 0) ? 4 : ((ITEMS % 2 == 0) ? 2 : 1);   // epilogue passes (BM/EP rows each)

    // dynamic LDS: STAGES K buffers (1 when K fits one tile) | the f32 epilogue tile, BM/EP rows at a time
    extern __shared__ __attribute__((aligned(16))) char smem[];

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid / WAVES_N, wn = wid % WAVES_N;

    // XCD-aware bijective remap (blocks b, b+8, ... share an XCD).
    const int nwg = gridDim.x, bid = blockIdx.x;
    const int q = nwg >> 3, r8 = nwg & 7, xcd = bid & 7;
    const int wg = (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + (bid >> 3);
    const int tn = wg % a.ntiles_n, tm = wg / a.ntiles_n;
    const int m0 = tm * BM, n0 = tn * BN;

    // ---- per-thread A-row decomposition (fixed across K) ----
    const int chunk = tid & 7, rbase = tid >> 3;
    // per A row: input position at tap (0,0) and its element offset there (may
    // point before the image; dereferenced only when the tap is inside)
    long pix0[A_IT];
    int iy0[A_IT], ix0[A_IT];
    const int ohw = a.yh * a.yw;
#pragma unroll
    for (int i = 0; i < A_IT; ++i) {
        int m = m0 + rbase + ROWS * i;
        if (m < a.M) {
            int b = m / ohw, rem = m - b * ohw;
            int oy = rem / a.yw, ox = rem - oy * a.yw;
            iy0[i] = oy * a.stride - a.pad;
            ix0[i] = ox * a.stride - a.pad;
            pix0[i] = (((long)b * a.xh + iy0[i]) * a.xw + ix0[i]) * a.ldx + a.xcoff;
        } else {
            iy0[i] = -(1 << 28); ix0[i] = 0; pix0[i] = 0;
        }
    }
    const long tap_dy = (long)a.xw * a.ldx;   // element offset of one tap row
    const T* wbase = (const T*)a.w + (size_t)(n0 + rbase) * a.kpad + chunk * VEC;

    u32x4 ra[A_IT], rb[B_IT];
    const int nk = a.kpad / BKE;
    const int cvec = a.cin_pad / VEC, ntap = a.kh * a.kw;

    // DENSE: whole tile inside one tap; track (kh, kw, c) incrementally.
    int t_kh = 0, t_kw = 0, t_c = 0;
    const T* xsafe = (const T*)a.x;

    // LDS-DMA form: every lane DMAs its 16-B chunk straight into the K buffer.
    // The destination is lane-linear (wave w, instruction i -> rows w*8+32i ..
    // +7, slot = lane&7), so the XOR swizzle moves to the SOURCE: the lane
    // fetches logical chunk (lane&7) ^ swz(row) (rule: swizzle both sides or
    // neither). Padding taps read the zero page.
    const int lchunk = (tid & 7) ^ ((rbase >> 1) & 7);
    // LDS-DMA through buffer descriptors (buffer_load_dwordx4 ... lds): 32-bit
    // per-lane byte offsets; an offset past num_records reads zeros (conv padding).
    constexpr int ESZ = (int)sizeof(T);
    const long xbytes = (long)a.B * a.xh * a.xw * a.ldx * ESZ;
    const __amdgpu_buffer_rsrc_t rsrc_x =
        __builtin_amdgcn_make_buffer_rsrc((void*)a.x, 0, (int)(xbytes < 0x7fffffffL ? xbytes : 0x7fffffffL), 0x00020000);
    const __amdgpu_buffer_rsrc_t rsrc_w = __builtin_amdgcn_make_buffer_rsrc((void*)a.w, 0, 0x7fffffff, 0x00020000);
    const unsigned woff_g = (unsigned)(((long)(n0 + rbase) * a.kpad + lchunk * VEC) * ESZ);
#define VD_GLDS_TILE(kt, buf)                                                              \
    do {                                                                                  \
        int dy, dx, c;                                                                    \
        bool kval = true;                                                                 \
        if constexpr (DENSE) {                                                            \
            dy = t_kh; dx = t_kw; c = t_c + lchunk * VEC;                                 \
        } else {                                                                          \
            const int kv = (kt) * 8 + lchunk;                                             \
            const int tap = kv / cvec;                                                    \
            c = (kv - tap * cvec) * VEC;                                                  \
            kval = tap < ntap;                                                            \
            dy = tap / a.kw; dx = tap - dy * a.kw;                                        \
        }                                                                                 \
        char* As_ = smem + (buf) * BUF;                                                   \
        char* Bs_ = As_ + BM * 128;                                                       \
        const long toff = dy * tap_dy + (long)dx * a.ldx + c;                             \
        _Pragma("unroll") for (int i = 0; i < A_IT; ++i) {                                \
            const int iy = iy0[i] + dy, ix = ix0[i] + dx;                                 \
            const bool ok = kval && (unsigned)iy < (unsigned)a.xh && (unsigned)ix < (unsigned)a.xw; \
            const unsigned off = ok ? (unsigned)((pix0[i] + toff) * ESZ) : 0x80000000u;  \
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc_x, (lds_void_t*)(As_ + (wid * 8 + ROWS * i) * 128), 16, \
                                                     off, 0, 0, 0);                      \
        }                                                                                 \
        _Pragma("unroll") for (int i = 0; i < B_IT; ++i)                                  \
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc_w, (lds_void_t*)(Bs_ + (wid * 8 + ROWS * i) * 128), 16, \
                                                     woff_g + (unsigned)(ROWS * i * a.kpad * ESZ), \
                                                     (unsigned)((kt) * BKE * ESZ), 0, 0);  \
        if constexpr (DENSE) {                                                            \
            t_c += BKE;                                                                   \
            if (t_c >= a.cin_pad) { t_c = 0; if (++t_kw == a.kw) { t_kw = 0; ++t_kh; } } \
        }                                                                                 \
    } while (0)

    f32x4_t acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

    // one K tile of fragment reads + MFMAs from LDS buffer `buf`
#define VD_COMPUTE(buf)                                                                     \
    do {                                                                                  \
        const char* As = smem + (buf) * BUF;                                              \
        const char* Bs = As + BM * 128;                                                   \
        _Pragma("unroll") for (int ks = 0; ks < NKS; ++ks) {                              \
            const int ch = ks * 4 + (lane >> 4);                                          \
            u32x4 af[TM], bfr[TN];                                                        \
            _Pragma("unroll") for (int i = 0; i < TM; ++i)                                \
                af[i] = *(const u32x4*)(As + lds_off(wm * WTM + i * 16 + (lane & 15), ch)); \
            _Pragma("unroll") for (int j = 0; j < TN; ++j)                                \
                bfr[j] = *(const u32x4*)(Bs + lds_off(wn * WTN + j * 16 + (lane & 15), ch)); \
            _Pragma("unroll") for (int i = 0; i < TM; ++i)                                \
            _Pragma("unroll") for (int j = 0; j < TN; ++j) {                              \
                if constexpr (std::is_same<T, float>::value) {                            \
                    const float* fa = (const float*)&af[i];                               \
                    const float* fb = (const float*)&bfr[j];                              \
                    _Pragma("unroll") for (int e = 0; e < 4; ++e)                         \
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[e], fb[e], acc[i][j], 0, 0, 0); \
                } else if constexpr (std::is_same<T, _Float16>::value) {                  \
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(                   \
                        __builtin_bit_cast(f16x8_t, af[i]), __builtin_bit_cast(f16x8_t, bfr[j]), \
                        acc[i][j], 0, 0, 0);                                              \
                } else {                                                                  \
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(                  \
                        __builtin_bit_cast(bf16x8_t, af[i]), __builtin_bit_cast(bf16x8_t, bfr[j]), \
                        acc[i][j], 0, 0, 0);                                              \
                }                                                                         \
            }                                                                             \
        }                                                                                 \
    } while (0)

    // Residual prefetch: the epilogue's 16-B residual vectors are loaded now, so
    // their latency overlaps the K loop instead of following it (c3 / FPN convs).
    const bool vec_ok = ((a.cout & 7) == 0) && ((a.ldy & 7) == 0) && ((a.ycoff & 7) == 0) &&
                        (a.res_mode == VD_RES_NONE || (((a.res_ld | a.res_coff) & 7) == 0));
    // (bf16 only; the exact-f32 parity mode reads its residual in the epilogue)
    const bool pf = vec_ok && a.res_mode != VD_RES_NONE && !std::is_same<T, float>::value;
    u32x4 rpf[ITEMS];
#pragma unroll
    for (int q = 0; q < ITEMS; ++q) {
        const int it = tid + NT * q;
        const int m = m0 + it / CG, nb = n0 + (it % CG) * 8;
        const bool ok = pf && m < a.M && nb < a.cout;
        size_t roff = 0;
        if (ok) {
            if (a.res_up) {
                const int b = m / ohw, rem = m - b * ohw;
                const int oy = rem / a.yw, ox = rem - oy * a.yw;
                roff = ((size_t)(b * a.rh + (oy >> 1)) * a.rw + (ox >> 1)) * a.res_ld + a.res_coff + nb;
            } else {
                roff = (size_t)m * a.res_ld + a.res_coff + nb;
            }
        }
        const T* rp = ok ? (const T*)a.res + roff : xsafe;
        rpf[q] = *(const u32x4*)rp;
    }

    {
        // Two LDS buffers, tile kt+1 in flight while kt is consumed. Raw barriers
        // with counted vmcnt: __syncthreads() would add vmcnt(0) and drain the DMA.
        constexpr int LPT = A_IT + B_IT;                 // DMA instructions per lane per tile
        VD_GLDS_TILE(0, 0);
        if (nk > 1) VD_GLDS_TILE(1, 1);
        for (int kt = 0; kt < nk; ++kt) {
            if (kt + 1 < nk) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LPT) : "memory");
            else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            VD_COMPUTE(kt & 1);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            if (kt + 2 < nk) VD_GLDS_TILE(kt + 2, kt & 1);
        }
    }

    // ---- fused epilogue ----
    // The f32 accumulator tile goes through LDS BM/EP rows at a time
    // ([BM/EP][BN+4], conflict-free fragment writes); each thread then owns 8
    // consecutive channels of a row: 16-B (bf16) / 32-B (f32) stores coalesced
    // along the NHWC channel dimension, with the prefetched residual.
    float* ep = (float*)smem;
#pragma unroll
    for (int h = 0; h < EP; ++h) {
        if (h) __syncthreads();
#pragma unroll
        for (int i = 0; i < TM; ++i) {
            const int row0 = wm * WTM + i * 16;
            if (row0 / (BM / EP) != h) continue;
#pragma unroll
            for (int j = 0; j < TN; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    ep[(row0 - h * (BM / EP) + (lane >> 4) * 4 + r) * EPLD + wn * WTN + j * 16 + (lane & 15)] =
                        acc[i][j][r];
        }
        __syncthreads();
#pragma unroll
        for (int q = h * (ITEMS / EP); q < (h + 1) * (ITEMS / EP); ++q) {
            const int it = tid + NT * q;
            const int rr = it / CG, cg = it % CG;
            const int m = m0 + rr;
            const int nb = n0 + cg * 8;
            if (m >= a.M || nb >= a.cout) continue;
            const float* er = ep + (rr - h * (BM / EP)) * EPLD + cg * 8;
            const size_t yo = (size_t)m * a.ldy + a.ycoff + nb;
            if (vec_ok) {
                float v[8], rv[8];
                const float4 s0 = *(const float4*)(a.scale + nb), s1 = *(const float4*)(a.scale + nb + 4);
                const float4 h0 = *(const float4*)(a.shift + nb), h1 = *(const float4*)(a.shift + nb + 4);
                const float sc[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
                const float sh[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
                const float4 e0 = *(const float4*)er, e1 = *(const float4*)(er + 4);
                const float ev[8] = {e0.x, e0.y, e0.z, e0.w, e1.x, e1.y, e1.z, e1.w};
                if (pf) {
                    using H = typename std::conditional<std::is_same<T, float>::value, __bf16, T>::type;
                    typedef H t8_t __attribute__((ext_vector_type(8)));
                    const t8_t rb8 = __builtin_bit_cast(t8_t, rpf[q]);
#pragma unroll
                    for (int e = 0; e < 8; ++e) rv[e] = (float)rb8[e];
                } else if (a.res_mode != VD_RES_NONE) {   // f32 residual, read here
                    size_t roff;
                    if (a.res_up) {
                        const int b = m / ohw, rem = m - b * ohw;
                        const int oy = rem / a.yw, ox = rem - oy * a.yw;
                        roff = ((size_t)(b * a.rh + (oy >> 1)) * a.rw + (ox >> 1)) * a.res_ld + a.res_coff + nb;
                    } else {
                        roff = (size_t)m * a.res_ld + a.res_coff + nb;
                    }
#pragma unroll
                    for (int e = 0; e < 8; ++e) rv[e] = load_elem<T>(a.res, roff + e);
                }
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    float t = ev[e] * sc[e] + sh[e];
                    if (a.res_mode == VD_RES_PRE_ACT) t += rv[e];
                    t = act_apply(t, a.act, a.slope);
                    if (a.res_mode == VD_RES_POST_ACT) t += rv[e];
                    v[e] = t;
                }
                if (a.out_f32 || std::is_same<T, float>::value) {
                    *(float4*)((float*)a.y + yo) = make_float4(v[0], v[1], v[2], v[3]);
                    *(float4*)((float*)a.y + yo + 4) = make_float4(v[4], v[5], v[6], v[7]);
                } else {
                    using H = typename std::conditional<std::is_same<T, float>::value, __bf16, T>::type;
                    typedef H t8_t __attribute__((ext_vector_type(8)));
                    t8_t o;
#pragma unroll
                    for (int e = 0; e < 8; ++e) o[e] = (H)v[e];
                    *(t8_t*)((H*)a.y + yo) = o;
                }
            } else {
                size_t roff = 0;
                if (a.res_mode != VD_RES_NONE) {
                    if (a.res_up) {
                        const int b = m / ohw, rem = m - b * ohw;
                        const int oy = rem / a.yw, ox = rem - oy * a.yw;
                        roff = ((size_t)(b * a.rh + (oy >> 1)) * a.rw + (ox >> 1)) * a.res_ld + a.res_coff;
                    } else {
                        roff = (size_t)m * a.res_ld + a.res_coff;
                    }
                }
                for (int e = 0; e < 8 && nb + e < a.cout; ++e) {
                    const int n = nb + e;
                    float t = er[e] * a.scale[n] + a.shift[n];
                    const float rv = a.res_mode != VD_RES_NONE ? load_elem<T>(a.res, roff + n) : 0.f;
                    if (a.res_mode == VD_RES_PRE_ACT) t += rv;
                    t = act_apply(t, a.act, a.slope);
                    if (a.res_mode == VD_RES_POST_ACT) t += rv;
                    if (a.out_f32 || std::is_same<T, float>::value) ((float*)a.y)[yo + e] = t;
                    else ((T*)a.y)[yo + e] = (T)t;
                }
            }
        }
    }
}

#undef VD_GLDS_TILE
#undef VD_COMPUTE

template <typename T, int BM, int BN, int NT = 256, int STAGES = 2>
hipError_t launch_bn(const ConvArgs& a0, bool dense, hipStream_t s) {
    ConvArgs a = a0;
    a.ntiles_n = (a.cout + BN - 1) / BN;
    const int mt = (a.M + BM - 1) / BM;
    dim3 grid(mt * a.ntiles_n), block(NT);
    constexpr int VEC = Elem<T>::VEC;
    constexpr int ITEMS = BM * (BN / 8) / NT, EP = (ITEMS % 4 == 0) ? 4 : ((ITEMS % 2 == 0) ? 2 : 1);   // as in the kernel
    constexpr size_t BUF = (size_t)(BM + BN) * 128, EPI = (size_t)(BM / EP) * (BN + 4) * 4;
    const int nk = a.kpad / (8 * VEC);
    const size_t lds = std::max((nk > 1 ? STAGES : 1) * BUF, EPI);
    if (dense) hipLaunchKernelGGL((conv_igemm_kernel<T, BM, BN, NT, 2, true>), grid, block, lds, s, a);
    else hipLaunchKernelGGL((conv_igemm_kernel<T, BM, BN, NT, 2, false>), grid, block, lds, s, a);
    return hipGetLastError();
}

}  // namespace

static const VdTune k_default_tune{};

// Tile selection: BN follows Cout (32 heads / 64 / 128 / 192), BM = 128 (64 when the
// 128-row grid is small); bf16 layers go to the streaming / phased / taps kernels
// where those apply. Weights must be packed with Npad a multiple of the chosen BN
// (runtime pads to 128).
hipError_t vd_launch_conv(const ConvArgs& a0, bool f32, hipStream_t s) {
    ConvArgs a = a0;
    if (!a.tune) a.tune = &k_default_tune;
    const VdTune& t = *a.tune;
    const int vec = f32 ? 4 : 8;
    const int bke = 8 * vec;
    const bool dense = (a.cin_pad % bke) == 0;
    if (a.x2) {   // fused conv3 + downsample: planned only where a dual streaming kernel applies
        if (f32) return vd_launch_conv_x6(a, s);
        if (!vd_conv1x1_dual_ok(a)) return hipErrorInvalidValue;
        return vd_launch_conv1x1_stream(a, s);
    }
    const int bn = a.cout <= 32 ? 32 : (a.cout <= 64 ? 64 : 128);
    const long tiles128 = (long)((a.M + 127) / 128) * ((a.cout + bn - 1) / bn);
    if (f32) {
        if (vd_conv_x6_ok(a)) return vd_launch_conv_x6(a, s);
        if (a.cout <= 32) return launch_bn<float, 128, 32>(a, dense, s);
        if (a.cout <= 64) return launch_bn<float, 128, 64>(a, dense, s);
        return launch_bn<float, 128, 128>(a, dense, s);
    }
    if (vd_conv1x1_stream_ok(a)) return vd_launch_conv1x1_stream(a, s);
    if (vd_conv_big_ok(a)) return vd_launch_conv_big(a, s);
    if (vd_conv_taps_ok(a)) return vd_launch_conv_taps(a, s);
    // Small grids (YOLO's deep levels, RetinaFace level 3): 64-row tiles give
    // twice the workgroups, so the launch covers more of the 256 CUs.
    // Cout 129-192 (the fused SSH conv5X5_1 + conv3X3): one 192-wide N tile instead
    // of two 128-wide ones, so each A tile is staged once.
    const bool n192 = a.cout > 128 && a.cout <= 192 && t.conv_n192;
    if (a.f16) {   // fp16 plan (VD_PREC_FP16): the same tiles on v_mfma_f32_16x16x32_f16
        if (tiles128 < t.conv_small) {
            if (n192) return launch_bn<_Float16, 64, 192>(a, dense, s);
            if (bn == 32) return launch_bn<_Float16, 64, 32>(a, dense, s);
            if (bn == 64) return launch_bn<_Float16, 64, 64>(a, dense, s);
            return launch_bn<_Float16, 64, 128>(a, dense, s);
        }
        if (bn == 32) return launch_bn<_Float16, 128, 32>(a, dense, s);
        if (bn == 64) return launch_bn<_Float16, 128, 64>(a, dense, s);
        if (n192) return launch_bn<_Float16, 128, 192>(a, dense, s);
        return launch_bn<_Float16, 128, 128>(a, dense, s);
    }
    if (tiles128 < t.conv_small) {
        if (n192) return launch_bn<__bf16, 64, 192>(a, dense, s);
        if (bn == 32) return launch_bn<__bf16, 64, 32>(a, dense, s);
        if (bn == 64) return launch_bn<__bf16, 64, 64>(a, dense, s);
        return launch_bn<__bf16, 64, 128>(a, dense, s);
    }
    if (bn == 32) return launch_bn<__bf16, 128, 32>(a, dense, s);
    if (bn == 64) return launch_bn<__bf16, 128, 64>(a, dense, s);
    if (n192) return launch_bn<__bf16, 128, 192>(a, dense, s);
    return launch_bn<__bf16, 128, 128>(a, dense, s);
}
