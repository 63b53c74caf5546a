// Access-pattern microbenchmark for the mosaic output pass: 64 frames of
// 1920x1080x3 bytes copied out of place by
//   0: grid-stride 4 x 16 B per thread (mosaic_copy_kernel's pattern)
//   1: band of R rows per workgroup, 48 B (16 pixels) per thread per iteration
//   2: as 1 with the next iteration's 48 B loaded before this one is stored
//   3: band of R rows, each wave copies contiguous 1 KB spans (16 B per lane)
//   hipcc -O3 --offload-arch=gfx950 tools/copybench.hip -o tools/copybench && tools/copybench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int N = 64, H = 1080, W = 1920, PITCH = W * 3;

__global__ __launch_bounds__(256) void k_grid(const uint4* s, uint4* d, size_t nv) {
    const size_t stride = (size_t)gridDim.x * 256;
    size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    for (; i + 3 * stride < nv; i += 4 * stride) {
        const uint4 v0 = s[i], v1 = s[i + stride], v2 = s[i + 2 * stride], v3 = s[i + 3 * stride];
        d[i] = v0; d[i + stride] = v1; d[i + 2 * stride] = v2; d[i + 3 * stride] = v3;
    }
    for (; i < nv; i += stride) d[i] = s[i];
}

template <int R>
__global__ __launch_bounds__(256) void k_band48(const uint8_t* in, uint8_t* out) {
    const int f = blockIdx.y, y0 = blockIdx.x * R;
    const int cpr = W / 16;
    const int rows = min(R, H - y0);
    for (int i = threadIdx.x; i < rows * cpr; i += 256) {
        const int r = i / cpr, c = i - r * cpr;
        const size_t o = ((size_t)f * H + y0 + r) * PITCH + (size_t)c * 48;
        const uint4* s4 = (const uint4*)(in + o);
        uint4* d4 = (uint4*)(out + o);
        const uint4 v0 = s4[0], v1 = s4[1], v2 = s4[2];
        d4[0] = v0; d4[1] = v1; d4[2] = v2;
    }
}

template <int R>
__global__ __launch_bounds__(256) void k_band48_pf(const uint8_t* in, uint8_t* out) {
    const int f = blockIdx.y, y0 = blockIdx.x * R;
    const int cpr = W / 16;
    const int rows = min(R, H - y0);
    const int tot = rows * cpr;
    auto off = [&](int i) { const int r = i / cpr, c = i - r * cpr; return ((size_t)f * H + y0 + r) * PITCH + (size_t)c * 48; };
    int i = threadIdx.x;
    if (i >= tot) return;
    size_t o = off(i);
    uint4 v0 = ((const uint4*)(in + o))[0], v1 = ((const uint4*)(in + o))[1], v2 = ((const uint4*)(in + o))[2];
    for (;;) {
        const int in2 = i + 256;
        uint4 n0{}, n1{}, n2{};
        size_t o2 = 0;
        if (in2 < tot) {
            o2 = off(in2);
            n0 = ((const uint4*)(in + o2))[0]; n1 = ((const uint4*)(in + o2))[1]; n2 = ((const uint4*)(in + o2))[2];
        }
        uint4* d4 = (uint4*)(out + o);
        d4[0] = v0; d4[1] = v1; d4[2] = v2;
        if (in2 >= tot) break;
        i = in2; o = o2; v0 = n0; v1 = n1; v2 = n2;
    }
}

template <int R>
__global__ __launch_bounds__(256) void k_band_lin(const uint8_t* in, uint8_t* out) {
    const int f = blockIdx.y, y0 = blockIdx.x * R;
    const int rows = min(R, H - y0);
    const size_t base = ((size_t)f * H + y0) * PITCH;
    const int nv = rows * PITCH / 16;
    const uint4* s4 = (const uint4*)(in + base);
    uint4* d4 = (uint4*)(out + base);
    int i = threadIdx.x;
    for (; i + 768 < nv; i += 1024) {
        const uint4 a = s4[i], b = s4[i + 256], c = s4[i + 512], d = s4[i + 768];
        d4[i] = a; d4[i + 256] = b; d4[i + 512] = c; d4[i + 768] = d;
    }
    for (; i < nv; i += 256) d4[i] = s4[i];
}

int main() {
    const size_t bytes = (size_t)N * H * PITCH;
    uint8_t *in, *out;
    hipMalloc(&in, bytes); hipMalloc(&out, bytes);
    hipMemset(in, 7, bytes); hipMemset(out, 0, bytes);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    auto run = [&](const char* name, auto launch) {
        for (int i = 0; i < 5; ++i) launch();
        hipEventRecord(e0);
        const int it = 50;
        for (int i = 0; i < it; ++i) launch();
        hipEventRecord(e1); hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        const double us = ms * 1e3 / it;
        printf("%-22s %8.1f us  %7.1f GB/s\n", name, us, 2.0 * bytes / (us * 1e-6) / 1e9);
    };
    const size_t nv = bytes / 16;
    run("grid 4x16B", [&] { hipLaunchKernelGGL(k_grid, dim3(1024, 1), dim3(256), 0, 0, (const uint4*)in, (uint4*)out, nv); });
    run("grid 4x16B 4096", [&] { hipLaunchKernelGGL(k_grid, dim3(4096, 1), dim3(256), 0, 0, (const uint4*)in, (uint4*)out, nv); });
    run("band16 48B", [&] { hipLaunchKernelGGL(k_band48<16>, dim3((H + 15) / 16, N), dim3(256), 0, 0, in, out); });
    run("band32 48B", [&] { hipLaunchKernelGGL(k_band48<32>, dim3((H + 31) / 32, N), dim3(256), 0, 0, in, out); });
    run("band8 48B", [&] { hipLaunchKernelGGL(k_band48<8>, dim3((H + 7) / 8, N), dim3(256), 0, 0, in, out); });
    run("band16 48B pf", [&] { hipLaunchKernelGGL(k_band48_pf<16>, dim3((H + 15) / 16, N), dim3(256), 0, 0, in, out); });
    run("band32 48B pf", [&] { hipLaunchKernelGGL(k_band48_pf<32>, dim3((H + 31) / 32, N), dim3(256), 0, 0, in, out); });
    run("band16 lin", [&] { hipLaunchKernelGGL(k_band_lin<16>, dim3((H + 15) / 16, N), dim3(256), 0, 0, in, out); });
    run("band32 lin", [&] { hipLaunchKernelGGL(k_band_lin<32>, dim3((H + 31) / 32, N), dim3(256), 0, 0, in, out); });
    run("hipMemcpyDtoD", [&] { hipMemcpyAsync(out, in, bytes, hipMemcpyDeviceToDevice, 0); });
    return 0;
}
