// x6bench.cpp — time the fp32-plan conv launchers (fp16 pairs, vd_launch_conv_x6 through
// vd_launch_conv) of libvdmi.so on synthetic RetinaFace layers at B = 64, 640x640 input:
// f32 NHWC activations with per-frame range slots, weights packed by vd_pack_x3h, the
// layer's residual where the network has one. No Python, no host copies in the timed loop.
//
//   hipcc -O2 -std=c++17 --offload-arch=gfx950 tools/x6bench.cpp \
//         -Ivideo-desensitization_amd/csrc -Iinclude -Lvideo-desensitization_amd/vdmi -lvdmi \
//         -Wl,-rpath,$PWD/video-desensitization_amd/vdmi -o tools/x6bench
//   tools/x6bench [reps] [layer-substring|all] [tune=value ...]
// tune names: the VdTune fields listed in kTune below (kernel selection / experiments).
#include "vd_common.h"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#define CK(x)                                                                                      \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } \
    } while (0)

struct Layer { const char* name; int H, W, cin, cout, k, s, p, res; };

// RetinaFace-R50 fp32-plan convs (B = 64): input spatial dims of the conv
static const Layer kLayers[] = {
    {"l2.0.c1", 160, 160, 256, 128, 1, 1, 0, 0},  {"l2.1.c1", 80, 80, 512, 128, 1, 1, 0, 0},
    {"l2.1.c2", 80, 80, 128, 128, 3, 1, 1, 0},    {"l2.1.c3", 80, 80, 128, 512, 1, 1, 0, 1},
    {"l2.0.ds", 160, 160, 256, 512, 1, 2, 0, 0},  {"l2.0.c2", 160, 160, 128, 128, 3, 2, 1, 0},
    {"l3.0.c1", 80, 80, 512, 256, 1, 1, 0, 0},    {"l3.0.c2", 80, 80, 256, 256, 3, 2, 1, 0},
    {"l3.0.ds", 80, 80, 512, 1024, 1, 2, 0, 0},   {"l3.1.c1", 40, 40, 1024, 256, 1, 1, 0, 0},
    {"l3.1.c2", 40, 40, 256, 256, 3, 1, 1, 0},    {"l3.1.c3", 40, 40, 256, 1024, 1, 1, 0, 1},
    {"l4.0.c1", 40, 40, 1024, 512, 1, 1, 0, 0},   {"l4.0.ds", 40, 40, 1024, 2048, 1, 2, 0, 0},
    {"l4.1.c1", 20, 20, 2048, 512, 1, 1, 0, 0},   {"l4.1.c2", 20, 20, 512, 512, 3, 1, 1, 0},
    {"l4.1.c3", 20, 20, 512, 2048, 1, 1, 0, 1},   {"fpn.o1", 80, 80, 512, 256, 1, 1, 0, 0},
    {"fpn.o2", 40, 40, 1024, 256, 1, 1, 0, 0},    {"fpn.o3", 20, 20, 2048, 256, 1, 1, 0, 0},
    {"fpn.m1", 80, 80, 256, 256, 3, 1, 1, 0},     {"ssh0.c51", 80, 80, 256, 192, 3, 1, 1, 0},
    {"ssh0.c52", 80, 80, 64, 128, 3, 1, 1, 0},    {"ssh0.c73", 80, 80, 64, 64, 3, 1, 1, 0},
    {"ssh1.c52", 40, 40, 64, 128, 3, 1, 1, 0},   {"l4.0.c3", 20, 20, 512, 2048, 1, 1, 0, 1},
    {"l3.0.c3", 40, 40, 256, 1024, 1, 1, 0, 1},   {"l4.0.c2", 40, 40, 512, 512, 3, 2, 1, 0},
};

struct TuneField { const char* name; int VdTune::*f; };
static const TuneField kTune[] = {
    {"x6_stream", &VdTune::x6_stream},   {"x6_stream256", &VdTune::x6_stream256}, {"x6_bn256", &VdTune::x6_bn256},
    {"x6_mid", &VdTune::x6_mid},         {"x6_mf32", &VdTune::x6_mf32},           {"x6_tail", &VdTune::x6_tail},
    {"x6_halo", &VdTune::x6_halo},       {"x6_halo_s2", &VdTune::x6_halo_s2}, {"x6_adepth", &VdTune::x6_adepth},       {"x6_small_k", &VdTune::x6_small_k},
    {"x6_small_tiles", &VdTune::x6_small_tiles}, {"x6_gemm1x1", &VdTune::x6_gemm1x1}, {"x6_dbg", &VdTune::x6_dbg},
    {"x6_halo_tr", &VdTune::x6_halo_tr}, {"x6_halo_dma", &VdTune::x6_halo_dma}, {"x6_halo_pf", &VdTune::x6_halo_pf}, {"x6_gemm_pf", &VdTune::x6_gemm_pf}, {"x6_gemm_uni", &VdTune::x6_gemm_uni}, {"x6_halo_1b", &VdTune::x6_halo_1b}, {"x6_stream_rl", &VdTune::x6_stream_rl}, {"x6_tr_epi", &VdTune::x6_tr_epi}, {"x6_halo_n64", &VdTune::x6_halo_n64}, {"x6_one", &VdTune::x6_one},
};

static float frand(uint32_t& st) {
    st = st * 1664525u + 1013904223u;
    return ((st >> 8) & 0xffff) / 32768.0f - 1.0f;
}

static double run(const Layer& L, int B, int reps, const VdTune& tune, bool check) {
    const int oh = (L.H + 2 * L.p - L.k) / L.s + 1, ow = (L.W + 2 * L.p - L.k) / L.s + 1;
    const int kpad = (L.k * L.k * L.cin + 31) / 32 * 32, npad = (L.cout + 127) / 128 * 128;
    const size_t nx = (size_t)B * L.H * L.W * L.cin, ny = (size_t)B * oh * ow * L.cout;
    std::vector<float> hx(nx), hw((size_t)npad * kpad, 0.f);
    uint32_t st = 12345;
    for (auto& v : hx) v = fmaxf(frand(st), 0.f) * 3.0f;          // post-ReLU activations
    for (int n = 0; n < L.cout; ++n)
        for (int k = 0; k < L.k * L.k * L.cin; ++k) hw[(size_t)n * kpad + k] = frand(st) * 0.05f;
    std::vector<uint16_t> hp((size_t)npad * kpad * 2);
    std::vector<float> rinv(npad), sc(npad), sh(npad);
    vd_pack_x3h(hw.data(), npad, kpad, hp.data(), rinv.data());
    for (int n = 0; n < npad; ++n) { sc[n] = rinv[n]; sh[n] = 0.01f; }
    void *dx, *dw, *dy, *dr = nullptr;
    float *dsc, *dsh;
    unsigned *dxm, *dym;
    CK(hipMalloc(&dx, nx * 4)); CK(hipMalloc(&dw, hp.size() * 2)); CK(hipMalloc(&dy, ny * 4));
    CK(hipMalloc(&dsc, npad * 4)); CK(hipMalloc(&dsh, npad * 4));
    CK(hipMalloc(&dxm, B * 4)); CK(hipMalloc(&dym, B * 4));
    CK(hipMemcpy(dx, hx.data(), nx * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dw, hp.data(), hp.size() * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(dsc, sc.data(), npad * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dsh, sh.data(), npad * 4, hipMemcpyHostToDevice));
    std::vector<unsigned> xm(B);
    const float three = 3.0f;
    for (auto& v : xm) memcpy(&v, &three, 4);
    CK(hipMemcpy(dxm, xm.data(), B * 4, hipMemcpyHostToDevice));
    CK(hipMemset(dym, 0, B * 4));
    if (L.res) {
        CK(hipMalloc(&dr, ny * 4));
        CK(hipMemcpy(dr, hx.data(), std::min(nx, ny) * 4, hipMemcpyHostToDevice));
    }
    ConvArgs a{};
    a.x = dx; a.xh = L.H; a.xw = L.W; a.ldx = L.cin; a.xcoff = 0;
    a.w = dw; a.scale = dsc; a.shift = dsh;
    a.res = dr; a.res_ld = L.cout; a.res_coff = 0; a.res_up = 0; a.rh = oh; a.rw = ow;
    a.res_mode = L.res ? VD_RES_PRE_ACT : VD_RES_NONE;
    a.y = dy; a.yh = oh; a.yw = ow; a.ldy = L.cout; a.ycoff = 0;
    a.B = B; a.cin_pad = L.cin; a.cout = L.cout; a.kpad = kpad;
    a.kh = L.k; a.kw = L.k; a.stride = L.s; a.pad = L.p;
    a.M = B * oh * ow; a.act = VD_ACT_RELU; a.slope = 0.f; a.out_f32 = 1;
    a.tune = &tune;
    a.wx3 = dw; a.scale_x = dsc; a.f32_split = 2;
    a.xmax = dxm; a.ymax = dym;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    for (int i = 0; i < 2; ++i) CK(vd_launch_conv(a, true, 0));
    CK(hipDeviceSynchronize());
    double err = -1.0;
    if (check) {   // a few outputs against a double-precision dot product
        std::vector<float> hy(ny);
        CK(hipMemcpy(hy.data(), dy, ny * 4, hipMemcpyDeviceToHost));
        err = 0.0;
        uint32_t s2 = 777;
        for (int t = 0; t < 256; ++t) {
            s2 = s2 * 1664525u + 1013904223u;
            const size_t m = (size_t)(s2 >> 4) % ((size_t)a.M);
            s2 = s2 * 1664525u + 1013904223u;
            const int n = (int)((s2 >> 4) % L.cout);
            const int b = (int)(m / (oh * ow)), rem = (int)(m % (oh * ow)), oy = rem / ow, ox = rem % ow;
            double acc = 0.0, mag = 0.0;
            for (int dy = 0; dy < L.k; ++dy)
                for (int dx2 = 0; dx2 < L.k; ++dx2) {
                    const int iy = oy * L.s - L.p + dy, ix = ox * L.s - L.p + dx2;
                    if (iy < 0 || ix < 0 || iy >= L.H || ix >= L.W) continue;
                    for (int c = 0; c < L.cin; ++c) {
                        const double xv = hx[(((size_t)b * L.H + iy) * L.W + ix) * L.cin + c];
                        const double wv = hw[(size_t)n * kpad + (dy * L.k + dx2) * L.cin + c];
                        acc += xv * wv;
                        mag += fabs(xv * wv);
                    }
                }
            double v = acc + 0.01;
            if (L.res) v += hx[m * L.cout + n < nx ? m * L.cout + n : 0];
            v = v > 0 ? v : 0;
            const double e = fabs(v - hy[m * L.cout + n]) / (mag + 1e-3);
            if (e > err) err = e;
        }
    }
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < reps; ++i) CK(vd_launch_conv(a, true, 0));
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / reps;
    const double fl = 2.0 * a.M * L.cout * (double)L.k * L.k * L.cin;
    printf("%-9s M=%8d N=%5d K=%5d  %8.1f us  %7.1f TF/s", L.name, a.M, L.cout, L.k * L.k * L.cin, us, fl / us * 1e-6);
    if (check) printf("  relerr %.2e", err);
    printf("\n");
    fflush(stdout);
    CK(hipFree(dx)); CK(hipFree(dw)); CK(hipFree(dy)); CK(hipFree(dsc)); CK(hipFree(dsh));
    CK(hipFree(dxm)); CK(hipFree(dym));
    if (dr) CK(hipFree(dr));
    return us;
}

int main(int argc, char** argv) {
    int reps = argc > 1 ? atoi(argv[1]) : 20;
    const std::string sel = argc > 2 ? argv[2] : "all";
    VdTune tune;
    bool check = getenv("X6_CHECK") != nullptr;
    for (int i = 3; i < argc; ++i) {
        const char* eq = strchr(argv[i], '=');
        if (!eq) { fprintf(stderr, "bad option %s\n", argv[i]); return 2; }
        const std::string k(argv[i], eq - argv[i]);
        bool ok = false;
        for (const TuneField& t : kTune)
            if (k == t.name) { tune.*(t.f) = atoi(eq + 1); ok = true; }
        if (!ok) { fprintf(stderr, "unknown option %s\n", k.c_str()); return 2; }
    }
    double tot = 0;
    for (const Layer& L : kLayers) {
        if (sel != "all" && std::string(L.name).find(sel) == std::string::npos) continue;
        tot += run(L, 64, reps, tune, check);
    }
    printf("total %.1f us\n", tot);
    return 0;
}
