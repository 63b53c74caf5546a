// convbench.cpp — time the conv launchers of libvdmi.so on synthetic bf16 layers
// (no Python, no host copies in the timed loop). Kernel choice is the library's
// default plan (VdTune defaults; ConvArgs.tune may point at a modified copy).
//
//   hipcc -O2 -std=c++17 --offload-arch=gfx950 tools/convbench.cpp \
//         -Ivideo-desensitization_amd/csrc -Iinclude -Lvideo-desensitization_amd/vdmi -lvdmi \
//         -Wl,-rpath,$PWD/video-desensitization_amd/vdmi -o tools/convbench
//   tools/convbench [reps]                      (built-in RetinaFace layer list, B=64)
//   tools/convbench reps B H W Cin Cout k s p   (one layer)
#include "vd_common.h"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#define CK(x)                                                                            \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } \
    } while (0)

struct Layer { const char* name; int B, H, W, cin, cout, k, s, p, res; };

static uint16_t f2bf(float f) {
    uint32_t u;
    memcpy(&u, &f, 4);
    return (uint16_t)((u + 0x7fff + ((u >> 16) & 1)) >> 16);
}

static double run(const Layer& L, int reps) {
    const int oh = (L.H + 2 * L.p - L.k) / L.s + 1, ow = (L.W + 2 * L.p - L.k) / L.s + 1;
    const int kpad = (L.k * L.k * L.cin + 63) / 64 * 64, npad = (L.cout + 255) / 256 * 256;
    const size_t nx = (size_t)L.B * L.H * L.W * L.cin, nw = (size_t)npad * kpad, ny = (size_t)L.B * oh * ow * L.cout;
    std::vector<uint16_t> hx(nx), hw(nw);
    uint32_t st = 12345;
    auto rnd = [&]() { st = st * 1664525u + 1013904223u; return ((st >> 8) & 0xffff) / 32768.0f - 1.0f; };
    for (auto& v : hx) v = f2bf(rnd());
    for (auto& v : hw) v = f2bf(rnd() * 0.05f);
    std::vector<float> sc(npad, 1.0f), sh(npad, 0.01f);
    void *dx, *dw, *dy, *dr = nullptr;
    float *dsc, *dsh;
    CK(hipMalloc(&dx, nx * 2)); CK(hipMalloc(&dw, nw * 2)); CK(hipMalloc(&dy, ny * 2));
    CK(hipMalloc(&dsc, npad * 4)); CK(hipMalloc(&dsh, npad * 4));
    CK(hipMemcpy(dx, hx.data(), nx * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(dw, hw.data(), nw * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(dsc, sc.data(), npad * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dsh, sh.data(), npad * 4, hipMemcpyHostToDevice));
    if (L.res) { CK(hipMalloc(&dr, ny * 2)); CK(hipMemset(dr, 0, ny * 2)); }
    ConvArgs a{};
    a.x = dx; a.xh = L.H; a.xw = L.W; a.ldx = L.cin; a.xcoff = 0;
    a.w = dw; a.scale = dsc; a.shift = dsh;
    a.res = dr; a.res_ld = L.cout; a.res_coff = 0; a.res_up = 0; a.rh = oh; a.rw = ow;
    a.res_mode = L.res ? VD_RES_PRE_ACT : VD_RES_NONE;
    a.y = dy; a.yh = oh; a.yw = ow; a.ldy = L.cout; a.ycoff = 0;
    a.B = L.B; a.cin_pad = L.cin; a.cout = L.cout; a.kpad = kpad;
    a.kh = L.k; a.kw = L.k; a.stride = L.s; a.pad = L.p;
    a.M = L.B * oh * ow; a.act = VD_ACT_RELU; a.slope = 0.f; a.out_f32 = 0;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    for (int i = 0; i < 3; ++i) CK(vd_launch_conv(a, false, 0));
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < reps; ++i) CK(vd_launch_conv(a, false, 0));
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / reps;
    const double fl = 2.0 * a.M * L.cout * (double)L.k * L.k * L.cin;
    printf("%-10s M=%8d N=%5d K=%5d  %8.1f us  %7.1f TF/s\n", L.name, a.M, L.cout, L.k * L.k * L.cin, us,
           fl / us * 1e-6);
    CK(hipFree(dx)); CK(hipFree(dw)); CK(hipFree(dy)); CK(hipFree(dsc)); CK(hipFree(dsh));
    if (dr) CK(hipFree(dr));
    return us;
}

// fused layer1 bottleneck (block.hip) on random bf16 data: B x H x W x cin -> 256
static void run_block(int reps, int B, int H, int W, int cin, bool ds) {
    auto rnd_buf = [](size_t n, float sc) {
        std::vector<uint16_t> h(n);
        uint32_t st = 777u + (uint32_t)n;
        for (auto& v : h) { st = st * 1664525u + 1013904223u; v = f2bf((((st >> 8) & 0xffff) / 32768.0f - 1.0f) * sc); }
        void* d;
        CK(hipMalloc(&d, n * 2));
        CK(hipMemcpy(d, h.data(), n * 2, hipMemcpyHostToDevice));
        return d;
    };
    BlockArgs a{};
    a.x = rnd_buf((size_t)B * H * W * cin, 1.0f);
    CK(hipMalloc(&a.y, (size_t)B * H * W * 256 * 2));
    a.B = B; a.H = H; a.W = W; a.cin = cin; a.ds = ds;
    a.tiles_x = (W + 15) / 16; a.tiles_y = (H + 7) / 8;
    a.w1 = rnd_buf((size_t)cin * 64, 0.05f);
    a.w2 = rnd_buf((size_t)4 * 18 * 64 * 8, 0.05f);
    a.w3 = rnd_buf((size_t)4 * 4 * 2 * 64 * 8, 0.05f);
    a.wd = rnd_buf((size_t)4 * 4 * (cin / 32) * 64 * 8, 0.05f);
    std::vector<float> bn(1280, 0.5f);
    float* dbn;
    CK(hipMalloc(&dbn, bn.size() * 4));
    CK(hipMemcpy(dbn, bn.data(), bn.size() * 4, hipMemcpyHostToDevice));
    a.bn = dbn;
    unsigned long long* ddiag;
    CK(hipMalloc(&ddiag, 8 * sizeof(unsigned long long)));
    a.diag = getenv("VD_DIAG") ? ddiag : nullptr;
    a.mode = getenv("VD_BLOCK_MODE") ? atoi(getenv("VD_BLOCK_MODE")) : 0;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    for (int i = 0; i < 3; ++i) CK(vd_launch_block(a, 0));
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < reps; ++i) CK(vd_launch_block(a, 0));
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / reps, px = (double)B * H * W;
    const double fl = 2.0 * px * (cin * 64 + 576 * 64 + 64 * 256 + (ds ? cin * 256 : 0));
    const double by = px * (cin + 256) * 2.0;
    printf("block cin=%d ds=%d %dx%dx%d  %8.1f us  %7.1f TF/s  %7.1f GB/s (x + y)\n", cin, (int)ds, B, H, W, us,
           fl / us * 1e-6, by / us * 1e-3);
    if (a.diag) {   // last launch's per-segment cycle sums (workgroup 0, wave 0)
        unsigned long long d[8];
        CK(hipMemcpy(d, ddiag, sizeof d, hipMemcpyDeviceToHost));
        const char* nm[8] = {"wait x", "barrier0", "stage1", "barrier1", "stage2", "barrier2", "stage3", "loop"};
        unsigned long long tot = 0;
        for (int i = 0; i < 8; ++i) tot += d[i];
        for (int i = 0; i < 8; ++i) printf("   %-9s %10llu cycles %5.1f%%\n", nm[i], d[i], 100.0 * d[i] / (tot ? tot : 1));
    }
}

// fused stem + maxpool (stem.hip) on random bf16 data: B x 321 x 321 x 16 -> B x 160 x 160 x 64
static void run_stem(int reps, int B) {
    const int xh = 321, xw = 321, ph = 160, pw = 160;
    std::vector<uint16_t> hx((size_t)B * xh * xw * 16), hw(4 * 8 * 64 * 8);
    uint32_t st = 99u;
    for (auto& v : hx) { st = st * 1664525u + 1013904223u; v = f2bf(((st >> 8) & 0xffff) / 65536.0f); }
    for (auto& v : hw) { st = st * 1664525u + 1013904223u; v = f2bf((((st >> 8) & 0xffff) / 32768.0f - 1.0f) * 0.1f); }
    StemPoolArgs a{};
    void *dx, *dy, *dw;
    float *dsc, *dsh;
    CK(hipMalloc(&dx, hx.size() * 2)); CK(hipMalloc(&dy, (size_t)B * ph * pw * 64 * 2)); CK(hipMalloc(&dw, hw.size() * 2));
    CK(hipMalloc(&dsc, 64 * 4)); CK(hipMalloc(&dsh, 64 * 4));
    CK(hipMemcpy(dx, hx.data(), hx.size() * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(dw, hw.data(), hw.size() * 2, hipMemcpyHostToDevice));
    std::vector<float> one(64, 1.0f), zero(64, 0.0f);
    CK(hipMemcpy(dsc, one.data(), 256, hipMemcpyHostToDevice));
    CK(hipMemcpy(dsh, zero.data(), 256, hipMemcpyHostToDevice));
    a.x = dx; a.B = B; a.xh = xh; a.xw = xw; a.y = dy; a.ph = ph; a.pw = pw; a.wf = dw; a.scale = dsc; a.shift = dsh;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    for (int i = 0; i < 3; ++i) CK(vd_launch_stem_pool(a, 0));
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < reps; ++i) CK(vd_launch_stem_pool(a, 0));
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / reps, fl = 2.0 * B * 320.0 * 320 * 64 * 147;
    printf("stem+pool B=%d  %8.1f us  %7.1f TF/s (147-term)\n", B, us, fl / us * 1e-6);
}

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 20;
    if (argc == 3 && std::string(argv[2]) == "stem") {
        run_stem(reps, 64);
        return 0;
    }
    if (argc == 3 && std::string(argv[2]) == "block") {
        run_block(reps, 64, 160, 160, 64, true);
        run_block(reps, 64, 160, 160, 256, false);
        return 0;
    }
    std::vector<Layer> layers;
    if (argc == 3 && std::string(argv[2]) == "yolo") {   // YOLOv8n-like small-channel layers, 640x384 canvas
        layers = {
            {"y.m0", 64, 384, 640, 8, 16, 3, 2, 1, 0},    {"y.m1", 64, 192, 320, 16, 32, 3, 2, 1, 0},
            {"y.c2f1x1", 64, 96, 160, 32, 32, 1, 1, 0, 0}, {"y.c2fm", 64, 96, 160, 16, 16, 3, 1, 1, 0},
            {"y.m3", 64, 96, 160, 32, 64, 3, 2, 1, 0},    {"y.m4m", 64, 48, 80, 32, 32, 3, 1, 1, 0},
            {"y.m5", 64, 48, 80, 64, 128, 3, 2, 1, 0},    {"y.head3", 64, 48, 80, 64, 64, 3, 1, 1, 0},
            {"y.c2f48", 64, 48, 80, 192, 64, 1, 1, 0, 0}, {"f.l1c2", 64, 160, 160, 64, 64, 3, 1, 1, 0},
            {"f.ssh52", 64, 80, 80, 64, 64, 3, 1, 1, 0},
        };
    } else if (argc == 3 && std::string(argv[2]) == "k512") {   // 1x1 layers of the HBM-bound family
        layers = {
            {"l2.c1", 64, 80, 80, 512, 128, 1, 1, 0, 0},   {"l3.0.c1", 64, 80, 80, 512, 256, 1, 1, 0, 0},
            {"l3.0.ds", 64, 80, 80, 512, 1024, 1, 2, 0, 0}, {"l4.c3", 64, 20, 20, 512, 2048, 1, 1, 0, 1},
            {"l3.c3", 64, 40, 40, 256, 1024, 1, 1, 0, 1},   {"l2.c3", 64, 80, 80, 128, 512, 1, 1, 0, 1},
        };
    } else if (argc >= 10) {
        layers.push_back({"custom", atoi(argv[2]), atoi(argv[3]), atoi(argv[4]), atoi(argv[5]), atoi(argv[6]),
                          atoi(argv[7]), atoi(argv[8]), atoi(argv[9]), 0});
    } else {
        layers = {
            {"l1.c2", 64, 160, 160, 64, 64, 3, 1, 1, 0},    {"l2.c2", 64, 80, 80, 128, 128, 3, 1, 1, 0},
            {"l2.c1", 64, 80, 80, 512, 128, 1, 1, 0, 0},    {"l3.c1", 64, 40, 40, 1024, 256, 1, 1, 0, 0},
            {"l3.c2", 64, 40, 40, 256, 256, 3, 1, 1, 0},    {"l3.c3", 64, 40, 40, 256, 1024, 1, 1, 0, 1},
            {"l4.c1", 64, 20, 20, 2048, 512, 1, 1, 0, 0},   {"l4.c2", 64, 20, 20, 512, 512, 3, 1, 1, 0},
            {"l4.c3", 64, 20, 20, 512, 2048, 1, 1, 0, 1},   {"fpn.m1", 64, 80, 80, 256, 256, 3, 1, 1, 0},
            {"ssh0.c3", 64, 80, 80, 256, 128, 3, 1, 1, 0},  {"ssh0.c51", 64, 80, 80, 256, 64, 3, 1, 1, 0},
        };
    }
    for (const auto& L : layers) run(L, reps);
    return 0;
}
