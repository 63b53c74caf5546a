// stamps.cpp — diagnostic: segment timing of the staggered 256x256 conv kernel.
// Builds conv_big.hip with VD_STAMPS (s_memtime at each segment edge of every
// phase, workgroup 0, lane 0 of each wave) on a plain GEMM-shaped 1x1 conv and
// prints the median cycles of: L = fragment reads + DMA issue, W = vmcnt wait,
// X = first barrier, C = lgkmcnt + 16 MFMAs, Y = second barrier (to next phase).
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -DVD_STAMPS -Iinclude \
//         -Ivideo-desensitization_amd/csrc tools/stamps.cpp -o tools/stamps
#include "../video-desensitization_amd/csrc/conv_big.hip"

#include <algorithm>
#include <cstdio>
#include <vector>

int vd_set_error(int code, const char*, ...) { return code; }

int main(int argc, char** argv) {
    const int M = argc > 1 ? atoi(argv[1]) : 4096, N = argc > 2 ? atoi(argv[2]) : 4096,
              K = argc > 3 ? atoi(argv[3]) : 4096;
    void *x, *w, *y;
    float *sc, *sh;
    (void)hipMalloc(&x, (size_t)M * K * 2); (void)hipMalloc(&w, (size_t)N * K * 2); (void)hipMalloc(&y, (size_t)M * N * 2);
    (void)hipMalloc(&sc, N * 4); (void)hipMalloc(&sh, N * 4);
    std::vector<uint16_t> h((size_t)std::max(M, N) * K);
    uint32_t st = 1;
    for (auto& v : h) { st = st * 1664525u + 1013904223u; v = (uint16_t)(0x3c00 | ((st >> 9) & 0x3ff)) ^ ((st & 1) << 15); }
    (void)hipMemcpy(x, h.data(), (size_t)M * K * 2, hipMemcpyHostToDevice);
    (void)hipMemcpy(w, h.data(), (size_t)N * K * 2, hipMemcpyHostToDevice);
    (void)hipMemset(sc, 0, N * 4); (void)hipMemset(sh, 0, N * 4);
    ConvArgs a{};
    a.x = x; a.xh = 1; a.xw = M; a.ldx = K; a.w = w; a.scale = sc; a.shift = sh;
    a.y = y; a.yh = 1; a.yw = M; a.ldy = N; a.B = 1; a.cin_pad = K; a.cout = N; a.kpad = K;
    a.kh = a.kw = a.stride = 1; a.M = M; a.act = VD_ACT_NONE;
    for (int i = 0; i < 5; ++i) (void)vd_launch_conv_big(a, 0);
    (void)hipDeviceSynchronize();
    std::vector<unsigned long long> s(8 * 2048);
    (void)hipMemcpyFromSymbol(s.data(), HIP_SYMBOL(vd_stamps), s.size() * 8);
    const char* names[5] = {"L(read+issue)", "W(vmcnt)", "X(barrier)", "C(lgkm+mfma)", "Y(barrier)"};
    const int nph = K / 64 * 4;
    for (int wv : {0, 4}) {
        const unsigned long long* p = &s[wv * 2048];
        std::vector<long> seg[5];
        for (int ph = 8; ph < nph - 8 && (ph + 1) * 5 < 2048; ++ph) {
            const unsigned long long* q = p + ph * 5;
            for (int k = 0; k < 4; ++k) seg[k].push_back((long)(q[k + 1] - q[k]));
            seg[4].push_back((long)(q[5] - q[4]));
        }
        printf("wave %d (median shader cycles per phase):", wv);
        long tot = 0;
        for (int k = 0; k < 5; ++k) {
            auto v = seg[k];
            std::nth_element(v.begin(), v.begin() + v.size() / 2, v.end());
            printf("  %s %ld", names[k], v[v.size() / 2]);
            tot += v[v.size() / 2];
        }
        printf("  | sum %ld (16 MFMA = 256 issue cycles)\n", tot);
    }
    return 0;
}
