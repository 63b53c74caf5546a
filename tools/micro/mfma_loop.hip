// mfma_loop.hip -- microbenchmark of the fp16-pair conv main loop body on gfx950: 8 waves per
// workgroup (2 per SIMD), each a 64 x 128 wave tile (acc[4][8] f32x4 = 128 VGPRs), per K step
// 8 A-fragment + 16 B-fragment ds_read_b128 from LDS and 96 v_mfma_f32_16x16x32_f16 (three
// products per accumulator). No global memory in the loop. Variants (template V):
//   0  three products per accumulator back to back (the conv kernels' order)
//   1  product-major: product p for all four accumulators of a column block, then p + 1
//   2  as 1, B fragments of block j + 1 read before block j's MFMAs
//   3  operands in registers only (no LDS reads in the loop): the MFMA issue ceiling
//   4  as 0, B of block j + 1 read before block j's MFMAs (the round-6 PF schedule)
//   5  as 4, plus the halo kernel's per-step A addresses (tap shift, padding flags, halo swizzle)
//   6  as 5, plus one s_barrier per K step (after lgkmcnt(0), as the conv kernels)
//   7  as 6 with the A addresses of step s + 1 computed during step s
//   hipcc -O3 --offload-arch=gfx950 tools/micro/mfma_loop.hip -o tools/micro/mfma_loop
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

#define MF(a, b, c) __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0, 0)

template <int V>
__global__ __launch_bounds__(512, 2) void loop_kernel(float* out, int steps) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    // conv-like operands (fp16 pair planes of scaled f32): hi planes uniform in (-2^14, 2^14),
    // lo planes 2^-11 of that -- finite sums, the power draw of real data (DVFS), unlike
    // random bit patterns (NaN / Inf accumulators)
    for (int i = tid; i < 96 * 1024 / 16; i += 512) {
        const bool lo = (i * 16 / 16384) & 1;
        u32x4 v;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            unsigned hsh = (unsigned)(i * 8 + 2 * k) * 2654435761u;
            hsh ^= hsh >> 15; hsh *= 2246822519u; hsh ^= hsh >> 13;
            const float f0 = ((float)(hsh & 0xFFFF) / 32768.f - 1.f) * (lo ? 8.f : 16384.f);
            const float f1 = ((float)(hsh >> 16) / 32768.f - 1.f) * (lo ? 8.f : 16384.f);
            const _Float16 h0 = (_Float16)f0, h1 = (_Float16)f1;
            v[k] = (unsigned)__builtin_bit_cast(unsigned short, h0) | ((unsigned)__builtin_bit_cast(unsigned short, h1) << 16);
        }
        ((u32x4*)smem)[i] = v;
    }
    __syncthreads();
    f32x4 acc[4][8];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // the conv kernels' LDS images: 64-B rows, 16-B chunk swizzled by row bit 3 (conflict-free
    // ds_read_b128 for 16-row fragments); A planes at 0 / 16 KB (256 rows), B at 32 / 48 KB
    auto off = [&](int row) { return row * 64 + (((lane >> 4) ^ (((row >> 3) & 1) * 3)) << 4); };
    int ao[4], bo[8];
#pragma unroll
    for (int i = 0; i < 4; ++i) ao[i] = off((wid >> 1) * 64 + i * 16 + (lane & 15));
#pragma unroll
    for (int j = 0; j < 8; ++j) bo[j] = 32768 + off((wid & 1) * 128 + j * 16 + (lane & 15));
    u32x4 af[4][2], bs[8][2];
    // halo-style A rows (V >= 5): a 256-row tile of an 80-wide image, rows shifted per tap
    const int W = 80, HR = 256 + 2 * W + 2;
    int arow[4], aflg[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int r = (wid >> 1) * 64 + i * 16 + (lane & 15), y = (r / W) % 80, x = r % W;
        arow[i] = r + W + 1;
        aflg[i] = (y > 0 ? 1 : 0) | (y < 79 ? 2 : 0) | (x > 0 ? 4 : 0) | (x < W - 1 ? 8 : 0) | 16;
    }
    auto swzh = [&](int row) { return row * 64 + (((lane >> 4) ^ (((row >> 2) & 1) << 1)) << 4); };
    int nxt[4];
    auto addr = [&](int s, int (&o)[4]) {
        const int tap = s % 9, dy = tap / 3 - 1, dx = tap - (tap / 3) * 3 - 1;
        const int need = (dy < 0 ? 1 : 0) | (dy > 0 ? 2 : 0) | (dx < 0 ? 4 : 0) | (dx > 0 ? 8 : 0) | 16;
        const int shift = dy * W + dx;
#pragma unroll
        for (int i = 0; i < 4; ++i) o[i] = swzh((aflg[i] & need) == need ? arow[i] + shift : HR) % 16384;
    };
    if (V == 7) addr(0, nxt);
    if (V == 3) {
#pragma unroll
        for (int i = 0; i < 4; ++i) { af[i][0] = *(u32x4*)(smem + ao[i]); af[i][1] = *(u32x4*)(smem + ao[i] + 16384); }
    }
    for (int s = 0; s < steps; ++s) {
        asm volatile("" ::: "memory");                       // LDS may have changed: no hoisting
        if (V >= 6) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
        }
        int cur[4];
        if (V == 5 || V == 6) addr(s, cur);
        if (V == 7) {
#pragma unroll
            for (int i = 0; i < 4; ++i) cur[i] = nxt[i];
        }
        if (V != 3) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int o = V >= 5 ? cur[i] : ao[i];
                af[i][0] = *(const u32x4*)(smem + o);
                af[i][1] = *(const u32x4*)(smem + o + 16384);
            }
        }
        if (V == 7) addr(s + 1, nxt);
        if (V == 2 || V >= 4) {
            u32x4 bq[2][2];
            bq[0][0] = *(const u32x4*)(smem + bo[0]);
            bq[0][1] = *(const u32x4*)(smem + bo[0] + 16384);
            __builtin_amdgcn_sched_group_barrier(0x0100, 10, 0);
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                if (j + 1 < 8) {
                    bq[(j + 1) & 1][0] = *(const u32x4*)(smem + bo[j + 1]);
                    bq[(j + 1) & 1][1] = *(const u32x4*)(smem + bo[j + 1] + 16384);
                    __builtin_amdgcn_sched_group_barrier(0x0100, 2, 0);
                }
                if (V == 2) {
#pragma unroll
                    for (int i = 0; i < 4; ++i) acc[i][j] = MF(bq[j & 1][1], af[i][0], acc[i][j]);
#pragma unroll
                    for (int i = 0; i < 4; ++i) acc[i][j] = MF(bq[j & 1][0], af[i][1], acc[i][j]);
#pragma unroll
                    for (int i = 0; i < 4; ++i) acc[i][j] = MF(bq[j & 1][0], af[i][0], acc[i][j]);
                } else {
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        acc[i][j] = MF(bq[j & 1][1], af[i][0], acc[i][j]);
                        acc[i][j] = MF(bq[j & 1][0], af[i][1], acc[i][j]);
                        acc[i][j] = MF(bq[j & 1][0], af[i][0], acc[i][j]);
                    }
                }
                __builtin_amdgcn_sched_group_barrier(0x0008, 12, 0);
            }
        } else {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                u32x4 bf[2];
                if (V == 3) { bf[0] = af[j & 3][1]; bf[1] = af[(j + 1) & 3][0]; }
                else {
                    bf[0] = *(const u32x4*)(smem + bo[j]);
                    bf[1] = *(const u32x4*)(smem + bo[j] + 16384);
                }
                if (V == 1) {
#pragma unroll
                    for (int i = 0; i < 4; ++i) acc[i][j] = MF(bf[1], af[i][0], acc[i][j]);
#pragma unroll
                    for (int i = 0; i < 4; ++i) acc[i][j] = MF(bf[0], af[i][1], acc[i][j]);
#pragma unroll
                    for (int i = 0; i < 4; ++i) acc[i][j] = MF(bf[0], af[i][0], acc[i][j]);
                } else {
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        acc[i][j] = MF(bf[1], af[i][0], acc[i][j]);
                        acc[i][j] = MF(bf[0], af[i][1], acc[i][j]);
                        acc[i][j] = MF(bf[0], af[i][0], acc[i][j]);
                    }
                }
            }
        }
    }
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) t += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
    out[blockIdx.x * 512 + tid] = t;
}

template <int V>
static void run(float* out, int blocks, int steps) {
    hipFuncSetAttribute((const void*)loop_kernel<V>, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(loop_kernel<V>, dim3(blocks), dim3(512), 96 * 1024, 0, out, steps);
    hipEventRecord(e0);
    const int reps = 10;
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(loop_kernel<V>, dim3(blocks), dim3(512), 96 * 1024, 0, out, steps);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    const double flop = 2.0 * 16 * 16 * 32 * 96.0 * 8 * steps * blocks * reps;
    printf("V%d  %8.3f ms  %7.1f TF/s f16  (%.3f of 2.5 PF)\n", V, ms / reps, flop / (ms * 1e-3) / 1e12,
           flop / (ms * 1e-3) / 2.5e15);
}

int main(int argc, char** argv) {
    const int steps = argc > 1 ? atoi(argv[1]) : 2000;
    int cus = 256;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    float* out;
    hipMalloc(&out, (size_t)cus * 512 * 4);
    run<3>(out, cus, steps);
    run<0>(out, cus, steps);
    run<1>(out, cus, steps);
    run<2>(out, cus, steps);
    run<4>(out, cus, steps);
    run<5>(out, cus, steps);
    run<6>(out, cus, steps);
    run<7>(out, cus, steps);
    run<3>(out, cus, steps);
    run<4>(out, cus, steps);
    run<6>(out, cus, steps);
    return 0;
}
