// chain.hip — a ResNet bottleneck's conv3 and the NEXT bottleneck's conv1 in one
// streaming pass (layer2: 128 -> 512 -> 128 channels).
//
// torchvision Bottleneck [ext] as built from the reference's body.layer2.*
// weights (detect_face/retinaface.py:53-60):
//   out = relu(bn3(conv3(t2)) + x)          512 ch: this block's output (and the
//                                            next block's identity)
//   t1' = relu(bn1'(conv1'(out)))           128 ch: the next block's conv1
// The two-kernel plan writes `out` and reads it straight back (420 MB per 64
// frames at 80x80); here it is consumed on chip while it is written, so HBM sees
// t2, x, out and t1' once each. Same arithmetic as the streaming 1x1 kernel for
// each conv (bf16 operands, f32 MFMA accumulation in the same K order, BN as
// acc*scale + shift, residual before the ReLU, bf16 rounding of `out`): the
// results equal the two-kernel plan bit for bit.
//
// One persistent workgroup of 8 waves per CU walks groups of 16 pixels:
//   loads    t2 (16 x 256 B) and x (16 x 1 KB) of group i + D arrive by LDS-DMA
//            (buffer_load ... lds, 1 KB per instruction, 3 per wave per group)
//            into a ring of D + 1 slots while group i computes; source-side chunk
//            swizzle (the DMA writes lane-linear) keeps the fragment reads
//            conflict-free. No register prefetch, so the weights can stay in VGPRs.
//   stage A  wave w: out channels 64w .. 64w+63 (4 MFMA tiles x 4 k-steps of
//            v_mfma_f32_16x16x32_bf16, D^T = W3 . T2^T); W3 fragments stationary,
//            rows permuted so a lane ends with 8 consecutive channels (16-B
//            stores); BN + residual + ReLU, bf16. The lane's two 8-channel
//            fragments are exactly B-operand fragments of conv1' k-steps 2w and
//            2w+1 -> LDS exchange.
//   stage B  wave w: t1' channels 16w .. 16w+15 over all 16 k-steps (W1'
//            fragments stationary, B fragments from the exchange).
// vmcnt counts LDS-DMA, loads and stores together in issue order; every wave
// issues exactly 3 DMA and 3 store instructions per group (tails: the DMA
// re-reads the last pixel, stores go past the buffer's num_records and are
// dropped), so the wait for group i's DMA is a fixed count once the ring is full.
#include "vd_common.h"

#include <cstdlib>

namespace {

// s_barrier after this wave's LDS ops retire (no global-memory fence)
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) void lds_void_t;


constexpr int C_MID = 128, C_OUT = 512;   // layer2 widths
constexpr int D = 3;                      // groups in flight ahead of the computing one
constexpr int R = D + 1;                  // ring slots
constexpr int SLOT_T2 = 16 * 256;         // t2 rows of a group (4 KB)
constexpr int SLOT = SLOT_T2 + 16 * 1024; // + identity rows (16 KB)
// s_waitcnt vmcnt(N) with expcnt / lgkmcnt left alone (gfx9 encoding: vmcnt[3:0] | vmcnt[5:4] << 14)
constexpr int vmcnt_imm(int n) { return (n & 15) | ((n >> 4) << 14) | 0x0F70 & ~15; }

// F16: the fp16 plan (VD_PREC_FP16) on fp16 operands / activations
template <bool F16>
__global__ __launch_bounds__(512, 1) void chain_kernel(ChainArgs a) {
    using HT = Half16<F16>;
    typedef typename HT::T T;
    const auto mfma = [](const u32x4& x, const u32x4& y, const f32x4_t& c) { return HT::mfma(x, y, c); };
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* ring = smem;                                     // R x SLOT
    u32x4* xch = (u32x4*)(smem + R * SLOT);                // exchange [16 k-steps][64 lanes]
    char* lscratch = smem + R * SLOT + 16 * 1024;          // sink of the padding DMA slot (1 KB)

    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int p = lane & 15, q = lane >> 4;
    const int groups = (a.M + 15) / 16;
    const int G = gridDim.x;
    const int g0 = blockIdx.x;
    if (g0 >= groups) return;
    const int ng = (groups - g0 + G - 1) / G;             // groups of this workgroup

    // ---- stationary operands (issued before any DMA: the compiler's waits on them
    // then count only older ops and can only over-wait) ----
    float sc3[2][8], sh3[2][8];    // bn3 of the lane's 16 output channels
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            sc3[h][e] = a.sc3[64 * w + 32 * h + 8 * q + e];
            sh3[h][e] = a.sh3[64 * w + 32 * h + 8 * q + e];
        }
    u32x4 w3f[4][4];   // conv3: tile j row i = channel 64w + 32(j>>1) + 8(i>>2) + 4(j&1) + (i&3)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int ch = 64 * w + 32 * (j >> 1) + 8 * (p >> 2) + 4 * (j & 1) + (p & 3);
        const T* wp = (const T*)a.w3 + (size_t)ch * a.kpad3 + 8 * q;
#pragma unroll
        for (int s = 0; s < 4; ++s) w3f[j][s] = *(const u32x4*)(wp + 32 * s);
    }
    u32x4 w1f[16];     // conv1': row i = channel 16w + i, 16 k-steps
    {
        const T* wp = (const T*)a.w1 + (size_t)(16 * w + p) * a.kpad1 + 8 * q;
#pragma unroll
        for (int s = 0; s < 16; ++s) w1f[s] = *(const u32x4*)(wp + 32 * s);
    }
    float sc1[4], sh1[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        sc1[r] = a.sc1[16 * w + 4 * q + r];
        sh1[r] = a.sh1[16 * w + 4 * q + r];
    }

    const __amdgpu_buffer_rsrc_t rt = __builtin_amdgcn_make_buffer_rsrc((void*)a.t2, 0, 0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc((void*)a.res, 0, 0x7fffffff, 0x00020000);
    const unsigned ybytes = (unsigned)((size_t)a.M * C_OUT * 2), y2bytes = (unsigned)((size_t)a.M * C_MID * 2);
    const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc(a.y, 0, (int)ybytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t ry2 = __builtin_amdgcn_make_buffer_rsrc(a.y2, 0, (int)y2bytes, 0x00020000);

    // DMA of local group i into slot i % R: 16 identity rows (1 KB each, instruction k =
    // pixel k) and 4 t2 instructions (4 pixels each); wave w issues identity rows 2w,
    // 2w+1 and t2 instruction w (waves 4-7: a padding slot into the scratch line).
    // LDS position c of a row holds logical 16-B chunk c ^ (pixel & 15).
    auto issue = [&](int i) {
        const int g = g0 + i * G;
        char* slot = ring + (i % R) * SLOT;
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const int pp = 2 * w + k;
            const int m = min(g * 16 + pp, a.M - 1);
            const unsigned off = (unsigned)(m * 1024 + ((lane ^ pp) << 4));
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rr, (lds_void_t*)(slot + SLOT_T2 + pp * 1024), 16, off, 0, 0, 0);
        }
        const bool real = w < 4;
        const int pp = 4 * (w & 3) + (lane >> 4), c = lane & 15;
        const int m = min(g * 16 + pp, a.M - 1);
        const unsigned off = (unsigned)(m * 256 + ((c ^ pp) << 4));
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rt, (lds_void_t*)(real ? slot + (w & 3) * 1024 : lscratch), 16, off,
                                                 0, 0, 0);
    };
#pragma unroll
    for (int i = 0; i < D; ++i)
        if (i < ng) issue(i);
        else issue(ng - 1);            // keep the per-wave DMA count uniform (re-load the last group)

#pragma unroll 1
    for (int i = 0; i < ng; ++i) {
        const int g = g0 + i * G;
        // group i's DMA landed: ops younger than it = 3 * (D - 1) DMA of the prologue /
        // earlier iterations + 3 stores per finished iteration since
        if (i == 0) __builtin_amdgcn_s_waitcnt(vmcnt_imm(3 * (D - 1)));
        else if (i == 1) __builtin_amdgcn_s_waitcnt(vmcnt_imm(3 * (D - 1) + 3));
        else if (i == 2) __builtin_amdgcn_s_waitcnt(vmcnt_imm(3 * (D - 1) + 6));
        else __builtin_amdgcn_s_waitcnt(vmcnt_imm(3 + 6 * (D - 1)));
        // raw barriers: the fence of __syncthreads() would also retire the DMA just issued
        lds_barrier();
        issue(i + D < ng ? i + D : ng - 1);                // slot (i + D) % R = slot of i - 1, read before the barrier
        const char* slot = ring + (i % R) * SLOT;
        int li = p, qq = q;
        asm volatile("" : "+v"(li), "+v"(qq));
        // ---- stage A: out = relu(bn3(W3 . t2) + x), channels 64w .. +64 ----
        f32x4_t acc[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const u32x4 tf = *(const u32x4*)(slot + li * 256 + (((4 * s + qq) ^ li) << 4));
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[j] = mfma(w3f[j][s], tf, acc[j]);
        }
        const unsigned mrow = (unsigned)(g * 16 + li);
        const bool ok = (int)mrow < a.M;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int c = 64 * w + 32 * h + 8 * qq;
            const u32x4 rf = *(const u32x4*)(slot + SLOT_T2 + li * 1024 + (((8 * w + 4 * h + qq) ^ li) << 4));
            const f32x4_t& lo = acc[2 * h];
            const f32x4_t& hi = acc[2 * h + 1];
            const float* sc = sc3[h];
            const float* sh = sh3[h];
            const float v[8] = {lo[0] * sc[0] + sh[0], lo[1] * sc[1] + sh[1], lo[2] * sc[2] + sh[2], lo[3] * sc[3] + sh[3],
                                hi[0] * sc[4] + sh[4], hi[1] * sc[5] + sh[5], hi[2] * sc[6] + sh[6], hi[3] * sc[7] + sh[7]};
            typename HT::V8 o;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float t0 = v[2 * e] + HT::lo(rf[e]);
                const float t1 = v[2 * e + 1] + HT::hi(rf[e]);
                o[2 * e] = (T)(t0 > 0.f ? t0 : 0.f);
                o[2 * e + 1] = (T)(t1 > 0.f ? t1 : 0.f);
            }
            const u32x4 ou = __builtin_bit_cast(u32x4, o);
            const unsigned yoff = ok ? (mrow * (unsigned)a.ld_y + (unsigned)c) * 2u : 0x80000000u;
            __builtin_amdgcn_raw_buffer_store_b128(ou, ry, yoff, 0, 0);
            xch[(2 * w + h) * 64 + lane] = ou;
        }
        lds_barrier();
        // ---- stage B: t1' = relu(bn1'(W1' . out)), channels 16w .. +16 ----
        f32x4_t acc2 = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < 16; ++s) acc2 = mfma(w1f[s], xch[s * 64 + lane], acc2);
        T o2[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const float t = acc2[r] * sc1[r] + sh1[r];
            o2[r] = (T)(t > 0.f ? t : 0.f);
        }
        const unsigned y2off = ok ? (mrow * (unsigned)a.ld_y2 + (unsigned)(16 * w + 4 * qq)) * 2u : 0x80000000u;
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, o2), ry2, y2off, 0, 0);
    }
    __builtin_amdgcn_s_waitcnt(vmcnt_imm(0));   // the trailing padding DMAs land before the workgroup exits
}

}  // namespace

// Eligible: the layer2 shape (128 -> 512 -> 128), bf16, dense rows (t2 / identity / out /
// t1' with channel strides 128 / 512 / 512 / 128, so a group's rows are contiguous for
// the 1-KB DMA), byte offsets within 2^31 (option chain=0 keeps the two-kernel plan).
bool vd_chain_ok(int cmid, int cout, int kpad3, int kpad1, int ld_t2, int ld_res, int ld_y, int ld_y2, long M) {
    if (cmid != C_MID || cout != C_OUT || kpad3 < C_MID || kpad1 < C_OUT || (kpad3 | kpad1) & 7) return false;
    if (ld_t2 != C_MID || ld_res != C_OUT || ld_y != C_OUT || ld_y2 != C_MID) return false;
    return M > 0 && M * C_OUT * 2 < 0x7fffffffL;
}

hipError_t vd_launch_chain(const ChainArgs& a, hipStream_t s) {
    if (a.M <= 0) return hipSuccess;
    constexpr size_t lds = (size_t)R * SLOT + 16 * 1024 + 1024;
    static const int cus = [] {
        (void)hipFuncSetAttribute((const void*)chain_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        (void)hipFuncSetAttribute((const void*)chain_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        int dev = 0, n = 256;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
        return n > 0 ? n : 256;
    }();
    const int groups = (a.M + 15) / 16;
    const int grid = groups < cus ? groups : cus;   // persistent: one workgroup per CU
    if (a.f16) hipLaunchKernelGGL(chain_kernel<true>, dim3(grid), dim3(512), lds, s, a);
    else hipLaunchKernelGGL(chain_kernel<false>, dim3(grid), dim3(512), lds, s, a);
    return hipGetLastError();
}
