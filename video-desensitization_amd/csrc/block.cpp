// block.cpp — plans for the fused layer1 bottleneck (block.hip): eligibility,
// weight repacking from the per-conv bf16 weights (so the fused op multiplies
// exactly the same bf16 values as the conv-by-conv chain), execution, and the
// vdt_bottleneck test entry (fused and conv-by-conv on the same inputs).
#include "../../include/vdmi.h"
#include "nets.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

namespace {

// LDS row R of a 64-row weight image (MFMA tile j = R/16, row i = R%16) holds
// channel 32(j>>1) + 8(i>>2) + 4(j&1) + (i&3): tiles 2p and 2p+1 then give a lane
// 8 consecutive output channels (block.hip stage-1 / stage-3 epilogues).
int perm_row(int R) {
    const int j = R >> 4, i = R & 15;
    return 32 * (j >> 1) + 8 * (i >> 2) + 4 * (j & 1) + (i & 3);
}

int fetch(const Conv& cv, std::vector<uint16_t>& w, std::vector<float>& sc, std::vector<float>& sh) {
    w.resize((size_t)cv.npad * cv.kpad);
    sc.resize(cv.npad);
    sh.resize(cv.npad);
    VD_CHECK_HIP(hipMemcpy(w.data(), cv.w, w.size() * 2, hipMemcpyDeviceToHost));
    VD_CHECK_HIP(hipMemcpy(sc.data(), cv.scale, sc.size() * 4, hipMemcpyDeviceToHost));
    VD_CHECK_HIP(hipMemcpy(sh.data(), cv.shift, sh.size() * 4, hipMemcpyDeviceToHost));
    return VD_OK;
}

// MFMA A-operand fragments [group][k-step][lane][8]: lane l holds output channel
// row(group, l%16) and K elements 32s + 8(l/16) .. +8 (block.hip / stem.hip layout)
template <class Row>
std::vector<uint16_t> frags(const std::vector<uint16_t>& src, int kpad, int groups, int ks, Row row) {
    std::vector<uint16_t> f((size_t)groups * ks * 64 * 8);
    for (int q = 0; q < groups; ++q)
        for (int s = 0; s < ks; ++s)
            for (int l = 0; l < 64; ++l)
                for (int e = 0; e < 8; ++e)
                    f[(((size_t)q * ks + s) * 64 + l) * 8 + e] = src[(size_t)row(q, l & 15) * kpad + 32 * s + 8 * (l >> 4) + e];
    return f;
}

// 32-channel groups of two MFMA tiles, rows permuted so a lane ends with 8
// consecutive output channels
int perm32(int q, int i) { return 32 * (q >> 1) + perm_row(16 * (q & 1) + i); }

bool is_conv(const Conv& c, int cin, int cout, int k, int stride, int pad, int act) {
    return c.cin == cin && c.cin_pad == cin && c.cout == cout && c.kh == k && c.kw == k && c.stride == stride &&
           c.pad == pad && c.act == act;
}

}  // namespace

bool Ctx::block_ok(int c1, int c2, int c3, int cd, const Act& x) const {
    const bool ds = cd >= 0;
    const int cin = x.c;
    if (f32) {   // fp32 plan: the fp16-pair block (block32.hip), on pair-packed convs with range slots
        if (!tune.block_fuse32 || !x.f32 || !x.amax || !vd_block32_ok(cin, ds, x.h, x.w)) return false;
        for (int c : {c1, c2, c3, cd})
            if (c >= 0 && (convs[c].split != 2 || !convs[c].wx3 || !convs[c].scale_x)) return false;
    } else if (x.f32 || !tune.block_fuse || !vd_block_ok(cin, ds, x.h, x.w)) {
        return false;
    }
    if (!is_conv(convs[c1], cin, 64, 1, 1, 0, VD_ACT_RELU)) return false;
    if (!is_conv(convs[c2], 64, 64, 3, 1, 1, VD_ACT_RELU)) return false;
    if (!is_conv(convs[c3], 64, 256, 1, 1, 0, VD_ACT_RELU)) return false;
    if (ds && !is_conv(convs[cd], cin, 256, 1, 1, 0, VD_ACT_NONE)) return false;
    return true;
}

// fp16-pair planes of a pair-packed conv ([npad][kpad/32][2][32] on the device) ->
// host [2][npad][kpad], plus its BN scale (row scales folded) and shift
static int fetch_pair(const Conv& cv, std::vector<uint16_t>& pl, std::vector<float>& sc, std::vector<float>& sh) {
    const int nk = cv.kpad / 32;
    std::vector<uint16_t> wx((size_t)cv.npad * cv.kpad * 2);
    VD_CHECK_HIP(hipMemcpy(wx.data(), cv.wx3, wx.size() * 2, hipMemcpyDeviceToHost));
    pl.resize(wx.size());
    for (int p = 0; p < 2; ++p)
        for (int n = 0; n < cv.npad; ++n)
            for (int k = 0; k < cv.kpad; ++k)
                pl[((size_t)p * cv.npad + n) * cv.kpad + k] = wx[(((size_t)n * nk + k / 32) * 2 + p) * 32 + k % 32];
    sc.resize(cv.npad);
    sh.resize(cv.npad);
    VD_CHECK_HIP(hipMemcpy(sc.data(), cv.scale_x, sc.size() * 4, hipMemcpyDeviceToHost));
    VD_CHECK_HIP(hipMemcpy(sh.data(), cv.shift, sh.size() * 4, hipMemcpyDeviceToHost));
    return VD_OK;
}

// block32.hip layouts from the convs' own fp16 pairs (the fused op multiplies exactly
// the weight values of the conv-by-conv fp32 plan)
static int make_block32(Ctx& c, Block& bk) {
    const int cin = bk.cin;
    std::vector<uint16_t> w1, w2, w3, wd;
    std::vector<float> s1, h1, s2, h2, s3, h3, sd, hd;
    int rc;
    if ((rc = fetch_pair(c.convs[bk.c1], w1, s1, h1))) return rc;
    if ((rc = fetch_pair(c.convs[bk.c2], w2, s2, h2))) return rc;
    if ((rc = fetch_pair(c.convs[bk.c3], w3, s3, h3))) return rc;
    if (bk.ds && (rc = fetch_pair(c.convs[bk.cd], wd, sd, hd))) return rc;
    const Conv &C1 = c.convs[bk.c1], &C2 = c.convs[bk.c2], &C3 = c.convs[bk.c3];
    const Conv* CD = bk.ds ? &c.convs[bk.cd] : nullptr;
    auto at = [](const std::vector<uint16_t>& pl, const Conv& cv, int p, int n, int k) {
        return pl[((size_t)p * cv.npad + n) * cv.kpad + k];
    };
    // conv1: LDS image source [plane][ks][row = channel][32]
    std::vector<uint16_t> f1((size_t)2 * (cin / 32) * 64 * 32);
    for (int p = 0; p < 2; ++p)
        for (int ks = 0; ks < cin / 32; ++ks)
            for (int n = 0; n < 64; ++n)
                for (int e = 0; e < 32; ++e)
                    f1[(((size_t)p * (cin / 32) + ks) * 64 + n) * 32 + e] = at(w1, C1, p, n, 32 * ks + e);
    // conv2: [jn][hf][tap][plane][lane][8], lane l: channel 16 jn + l % 16, k = tap * 64 + 32 hf + 8 (l / 16) + e
    std::vector<uint16_t> f2((size_t)4 * 2 * 9 * 2 * 64 * 8);
    for (int jn = 0; jn < 4; ++jn)
        for (int hf = 0; hf < 2; ++hf)
            for (int tp = 0; tp < 9; ++tp)
                for (int p = 0; p < 2; ++p)
                    for (int l = 0; l < 64; ++l)
                        for (int e = 0; e < 8; ++e)
                            f2[(((((size_t)jn * 2 + hf) * 9 + tp) * 2 + p) * 64 + l) * 8 + e] =
                                at(w2, C2, p, 16 * jn + (l & 15), tp * 64 + 32 * hf + 8 * (l >> 4) + e);
    // conv3 / downsample: [wave][tile j][k-step s][plane][lane][8], rows permuted so that
    // a lane's tiles j = 0, 1 give it channels 32 w + 8 (l / 16) + 4 j + (0..3)
    auto f3frag = [&](const std::vector<uint16_t>& src, const Conv& cv) {
        std::vector<uint16_t> f((size_t)8 * 2 * 2 * 2 * 64 * 8);
        for (int w = 0; w < 8; ++w)
            for (int j = 0; j < 2; ++j)
                for (int s = 0; s < 2; ++s)
                    for (int p = 0; p < 2; ++p)
                        for (int l = 0; l < 64; ++l)
                            for (int e = 0; e < 8; ++e) {
                                const int i = l & 15;
                                const int n = 32 * w + 8 * (i >> 2) + 4 * j + (i & 3);
                                f[(((((size_t)w * 2 + j) * 2 + s) * 2 + p) * 64 + l) * 8 + e] =
                                    at(src, cv, p, n, 32 * s + 8 * (l >> 4) + e);
                            }
        return f;
    };
    std::vector<uint16_t> f3 = f3frag(w3, C3), fd;
    if (bk.ds) fd = f3frag(wd, *CD);
    std::vector<float> bn(256 + 512 * (bk.ds ? 2 : 1), 0.f);
    for (int k = 0; k < 64; ++k) {
        bn[k] = s1[k]; bn[64 + k] = h1[k]; bn[128 + k] = s2[k]; bn[192 + k] = h2[k];
    }
    for (int k = 0; k < 256; ++k) {
        bn[256 + k] = s3[k]; bn[512 + k] = h3[k];
        if (bk.ds) { bn[768 + k] = sd[k]; bn[1024 + k] = hd[k]; }
    }
    auto up = [&](void** dst, const void* src, size_t bytes) {
        int r = c.dalloc(dst, bytes);
        if (r) return r;
        VD_CHECK_HIP(hipMemcpy(*dst, src, bytes, hipMemcpyHostToDevice));
        return VD_OK;
    };
    if ((rc = up(&bk.w1, f1.data(), f1.size() * 2))) return rc;
    if ((rc = up(&bk.w2, f2.data(), f2.size() * 2))) return rc;
    if ((rc = up(&bk.w3, f3.data(), f3.size() * 2))) return rc;
    if (bk.ds && (rc = up(&bk.wd, fd.data(), fd.size() * 2))) return rc;
    if ((rc = up((void**)&bk.bn, bn.data(), bn.size() * 4))) return rc;
    bk.f32 = true;
    return VD_OK;
}

int Ctx::make_block(int c1, int c2, int c3, int cd, int* idx) {
    Block bk;
    bk.cin = convs[c1].cin;
    bk.ds = cd >= 0;
    bk.c1 = c1; bk.c2 = c2; bk.c3 = c3; bk.cd = cd;
    const int cin = bk.cin;
    std::vector<uint16_t> w1, w2, w3, wd;
    std::vector<float> s1, h1, s2, h2, s3, h3, sd, hd;
    int rc;
    if (f32) {
        if ((rc = make_block32(*this, bk))) return rc;
        blocks.push_back(bk);
        *idx = (int)blocks.size() - 1;
        return VD_OK;
    }
    if ((rc = fetch(convs[c1], w1, s1, h1))) return rc;
    if ((rc = fetch(convs[c2], w2, s2, h2))) return rc;
    if ((rc = fetch(convs[c3], w3, s3, h3))) return rc;
    if (bk.ds && (rc = fetch(convs[cd], wd, sd, hd))) return rc;
    const int k1 = convs[c1].kpad, k2 = convs[c2].kpad, k3 = convs[c3].kpad, kd = bk.ds ? convs[cd].kpad : 0;

    // conv1 / conv2: 16-channel groups (stage 1 / 2 wave columns); conv2's K order is
    // (tap, c) with 64 channels per tap, so k-step s = 32-channel half s&1 of tap s>>1
    const auto id16 = [](int q, int i) { return 16 * q + i; };
    std::vector<uint16_t> f1 = frags(w1, k1, 4, cin / 32, id16);
    std::vector<uint16_t> f2 = frags(w2, k2, 4, 18, id16);
    // conv3 / downsample: 32-channel groups of two tiles, rows permuted so a lane
    // ends with 8 consecutive output channels
    std::vector<uint16_t> f3 = frags(w3, k3, 16, 2, perm32), fd;
    if (bk.ds) fd = frags(wd, kd, 16, cin / 32, perm32);
    std::vector<float> bn(1280, 0.f);
    for (int c = 0; c < 64; ++c) {
        bn[c] = s1[c]; bn[64 + c] = h1[c]; bn[128 + c] = s2[c]; bn[192 + c] = h2[c];
    }
    for (int c = 0; c < 256; ++c) {
        bn[256 + c] = s3[c]; bn[512 + c] = h3[c];
        if (bk.ds) { bn[768 + c] = sd[c]; bn[1024 + c] = hd[c]; }
    }
    auto up = [&](void** dst, const void* src, size_t bytes) {
        int r = dalloc(dst, bytes);
        if (r) return r;
        VD_CHECK_HIP(hipMemcpy(*dst, src, bytes, hipMemcpyHostToDevice));
        return VD_OK;
    };
    if ((rc = up(&bk.w1, f1.data(), f1.size() * 2))) return rc;
    if ((rc = up(&bk.w2, f2.data(), f2.size() * 2))) return rc;
    if ((rc = up(&bk.w3, f3.data(), f3.size() * 2))) return rc;
    if (bk.ds && (rc = up(&bk.wd, fd.data(), fd.size() * 2))) return rc;
    if ((rc = up((void**)&bk.bn, bn.data(), bn.size() * 4))) return rc;
    blocks.push_back(bk);
    *idx = (int)blocks.size() - 1;
    return VD_OK;
}

int Ctx::add_block(Net& net, int bi, const Act& x, Act& y) {
    const Block& bk = blocks[bi];
    if (x.c != bk.cin || y.c != 256 || y.h != x.h || y.w != x.w || x.f32 != bk.f32 || y.f32 != bk.f32 ||
        (bk.f32 && (!x.amax || !y.amax)))
        return vd_set_error(VD_ERR_ARG, "fused bottleneck plan shape mismatch");
    Op op{};
    op.kind = OP_BLOCK;
    op.blk = bi;
    op.x = x;
    op.y = y;
    net.ops.push_back(op);
    return VD_OK;
}

// stem conv (space-to-depth 4x4, 16 -> 64) + maxpool 3x3/2 (stem.hip)
int Ctx::add_stem_pool(Net& net, int ci, const Act& x, Act& y) {
    const Conv& cv = convs[ci];
    const bool pair = f32 && cv.split == 2;             // fp32 plan: fp16 pair weights, f32 pooled map
    if ((f32 && !pair) || x.f32 || y.f32 != pair || (pair && !cv.wx3) || cv.cin != 16 || cv.cin_pad != 16 || cv.cout != 64 || cv.kh != 4 || cv.kw != 4 ||
        cv.stride != 1 || cv.pad != 1 || cv.act != VD_ACT_RELU || cv.kpad != 256 || x.c != 16 || y.c != 64 ||
        !vd_stem_pool_ok(x.h, x.w, y.h, y.w))
        return vd_set_error(VD_ERR_ARG, "fused stem plan shape mismatch");
    std::vector<uint16_t> f;
    int rc;
    if (pair) {   // planes of the packed pair [npad][kpad / 32][2][32] -> fragments, hi then lo
        const int nk = cv.kpad / 32;
        std::vector<uint16_t> wx((size_t)cv.npad * cv.kpad * 2), pl((size_t)cv.npad * cv.kpad);
        VD_CHECK_HIP(hipMemcpy(wx.data(), cv.wx3, wx.size() * 2, hipMemcpyDeviceToHost));
        for (int p = 0; p < 2; ++p) {
            for (int n = 0; n < cv.npad; ++n)
                for (int k = 0; k < cv.kpad; ++k)
                    pl[(size_t)n * cv.kpad + k] = wx[(((size_t)n * nk + k / 32) * 2 + p) * 32 + k % 32];
            std::vector<uint16_t> fp = frags(pl, cv.kpad, 4, 8, perm32);
            f.insert(f.end(), fp.begin(), fp.end());
        }
    } else {
        std::vector<uint16_t> w;
        std::vector<float> sc, sh;
        if ((rc = fetch(cv, w, sc, sh))) return rc;
        f = frags(w, cv.kpad, 4, 8, perm32);
    }
    Op op{};
    op.kind = OP_STEMPOOL;
    op.conv = ci;
    op.x = x;
    op.y = y;
    if ((rc = dalloc(&op.wf, f.size() * 2))) return rc;
    VD_CHECK_HIP(hipMemcpy(op.wf, f.data(), f.size() * 2, hipMemcpyHostToDevice));
    net.ops.push_back(op);
    return VD_OK;
}

static inline const void* foff_b(const Act& a, int f0) {
    return (const char*)a.p + (size_t)f0 * a.h * a.w * a.c * 2;
}

int Ctx::run_block_op(const Op& op, int f0, int n, int fam) {
    const Block& bk = blocks[op.blk];
    double fpp = convs[bk.c1].flops_per_px + convs[bk.c2].flops_per_px + convs[bk.c3].flops_per_px;
    if (bk.ds) fpp += convs[bk.cd].flops_per_px;
    if (bk.f32) {
        Block32Args a{};
        a.x = (const char*)op.x.p + (size_t)f0 * op.x.h * op.x.w * op.x.c * 4;
        a.y = (char*)op.y.p + (size_t)f0 * op.y.h * op.y.w * op.y.c * 4;
        a.B = n; a.H = op.x.h; a.W = op.x.w; a.cin = bk.cin; a.ds = bk.ds;
        a.tiles_x = (a.W + 15) / 16;
        a.tiles_y = (a.H + 7) / 8;
        a.w1 = bk.w1; a.w2 = bk.w2; a.w3 = bk.w3; a.wd = bk.wd; a.bn = bk.bn;
        a.xmax = op.x.amax + f0;
        a.ymax = op.y.amax + f0;
        a.xdepth = tune.block32_xd;
        a.pipe = tune.block32_pipe;
        a.dbg = tune.block32_dbg;
        t_begin(fam, fpp * n * a.H * a.W);
        hipError_t e = vd_launch_block32(a, stream);
        t_end();
        if (e != hipSuccess) return vd_set_error(VD_ERR_HIP, "fused fp32 bottleneck launch: %s", hipGetErrorString(e));
        return VD_OK;
    }
    BlockArgs a{};
    a.x = foff_b(op.x, f0);
    a.y = (void*)foff_b(op.y, f0);
    a.B = n; a.H = op.x.h; a.W = op.x.w; a.cin = bk.cin; a.ds = bk.ds;
    a.tiles_x = (a.W + 15) / 16;
    a.tiles_y = (a.H + 7) / 8;
    a.w1 = bk.w1; a.w2 = bk.w2; a.w3 = bk.w3; a.wd = bk.wd; a.bn = bk.bn;
    a.f16 = f16 ? 1 : 0;
    t_begin(fam, fpp * n * a.H * a.W);
    hipError_t e = vd_launch_block(a, stream);
    t_end();
    if (e != hipSuccess) return vd_set_error(VD_ERR_HIP, "fused bottleneck launch: %s", hipGetErrorString(e));
    return VD_OK;
}

int Ctx::run_stem_pool_op(const Op& op, int f0, int n, int fam) {
    const Conv& cv = convs[op.conv];
    StemPoolArgs a{};
    a.x = foff_b(op.x, f0); a.B = n; a.xh = op.x.h; a.xw = op.x.w;
    a.y = (void*)((char*)op.y.p + (size_t)f0 * op.y.h * op.y.w * op.y.c * (op.y.f32 ? 4 : 2)); a.ph = op.y.h; a.pw = op.y.w;
    a.wf = op.wf; a.scale = cv.scale; a.shift = cv.shift;
    a.f16 = f16 ? 1 : 0;
    const bool pair = op.y.f32;
    if (pair) {
        a.scale = cv.scale_x;                           // BN scale with the weights' power-of-two folded in
        a.ymax = op.y.amax ? op.y.amax + f0 : nullptr;
    }
    t_begin(fam, cv.flops_per_px * n * (double)(op.x.h - 1) * (op.x.w - 1));
    hipError_t e = pair ? vd_launch_stem_pool32(a, stream) : vd_launch_stem_pool(a, stream);
    t_end();
    if (e != hipSuccess) return vd_set_error(VD_ERR_HIP, "fused stem launch: %s", hipGetErrorString(e));
    return VD_OK;
}

static uint16_t bf16_rne(float f) {
    uint32_t u;
    memcpy(&u, &f, 4);
    if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);
    u += 0x7fffu + ((u >> 16) & 1u);
    return (uint16_t)(u >> 16);
}

extern "C" int vdt_bottleneck(vd_ctx* h, const float* x, int n, int hh, int ww, int cin, const float* w1,
                              const float* bn1, const float* w2, const float* bn2, const float* w3, const float* bn3,
                              const float* wd, const float* bnd, int fused, float* y) {
    Ctx* ctx = (Ctx*)h;
    if (!ctx) return vd_set_error(VD_ERR_ARG, "null context");
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (hipSetDevice(ctx->device) != hipSuccess) return vd_set_error(VD_ERR_HIP, "hipSetDevice failed");
    if (ctx->f16 || (ctx->f32 && ctx->tune.f32_split != 2))
        return vd_set_error(VD_ERR_ARG, "vdt_bottleneck: bf16 or fp32 (fp16-pair) contexts only");
    const bool f32 = ctx->f32;
    if (n <= 0 || hh <= 0 || ww <= 0 || !x || !w1 || !w2 || !w3 || !bn1 || !bn2 || !bn3 || !y ||
        (cin != 64 && cin != 256) || (wd && !bnd) || (!wd && cin != 256))
        return vd_set_error(VD_ERR_ARG, "vdt_bottleneck: bad arguments");
    const size_t nalloc = ctx->allocs.size(), nconv = ctx->convs.size(), nblk = ctx->blocks.size();
    auto cleanup = [&]() {
        for (size_t i = nalloc; i < ctx->allocs.size(); ++i) hipFree(ctx->allocs[i]);
        ctx->allocs.resize(nalloc);
        ctx->convs.resize(nconv);
        ctx->blocks.resize(nblk);
    };
    auto mk = [&](const float* wt, const float* bn, int ci, int co, int k, int pad, int act, int* idx) {
        Conv cv{};
        cv.cin = ci; cv.cout = co; cv.kh = k; cv.kw = k; cv.stride = 1; cv.pad = pad; cv.act = act;
        std::vector<float> wv(wt, wt + (size_t)co * ci * k * k), sc(bn, bn + co), sh(bn + co, bn + 2 * co);
        int r = ctx->upload_conv(cv, wv, sc, sh);
        if (r) return r;
        ctx->convs.push_back(cv);
        *idx = (int)ctx->convs.size() - 1;
        return VD_OK;
    };
    int c1, c2, c3, cd = -1, rc;
    if ((rc = mk(w1, bn1, cin, 64, 1, 0, VD_ACT_RELU, &c1)) || (rc = mk(w2, bn2, 64, 64, 3, 1, VD_ACT_RELU, &c2)) ||
        (rc = mk(w3, bn3, 64, 256, 1, 0, VD_ACT_RELU, &c3)) || (wd && (rc = mk(wd, bnd, cin, 256, 1, 0, VD_ACT_NONE, &cd)))) {
        cleanup();
        return rc;
    }
    auto buf = [&](Act& a, int c) {
        a.h = hh; a.w = ww; a.c = c; a.f32 = f32;
        const size_t bytes = (size_t)n * hh * ww * c * (f32 ? 4 : 2);
        int r = ctx->dalloc(&a.p, bytes);
        if (!r && hipMemset(a.p, 0, bytes) != hipSuccess) r = vd_set_error(VD_ERR_HIP, "hipMemset");
        if (!r && f32) {   // per-frame range slots (zero: producers fold their maxima in)
            r = ctx->dalloc((void**)&a.amax, (size_t)n * 4);
            if (!r && hipMemset(a.amax, 0, (size_t)n * 4) != hipSuccess) r = vd_set_error(VD_ERR_HIP, "hipMemset");
        }
        return r;
    };
    Act ax, at1, at2, aout, ads;
    if ((rc = buf(ax, cin)) || (rc = buf(aout, 256))) { cleanup(); return rc; }
    if (f32) {   // f32 input and its per-frame max |x| (what its producer would have folded)
        const size_t fe = (size_t)hh * ww * cin;
        std::vector<unsigned> mx(n, 0u);
        for (int b = 0; b < n; ++b) {
            float m = 0.f;
            for (size_t i = 0; i < fe; ++i) m = std::max(m, std::fabs(x[b * fe + i]));
            memcpy(&mx[b], &m, 4);
        }
        if (hipMemcpy(ax.p, x, (size_t)n * fe * 4, hipMemcpyHostToDevice) != hipSuccess ||
            hipMemcpy(ax.amax, mx.data(), (size_t)n * 4, hipMemcpyHostToDevice) != hipSuccess) {
            cleanup();
            return vd_set_error(VD_ERR_HIP, "vdt_bottleneck: upload");
        }
    } else {
        std::vector<uint16_t> xb((size_t)n * hh * ww * cin);
        for (size_t i = 0; i < xb.size(); ++i) xb[i] = bf16_rne(x[i]);
        if (hipMemcpy(ax.p, xb.data(), xb.size() * 2, hipMemcpyHostToDevice) != hipSuccess) {
            cleanup();
            return vd_set_error(VD_ERR_HIP, "vdt_bottleneck: upload");
        }
    }
    Net net;
    if (fused) {
        int bi;
        if (!ctx->block_ok(c1, c2, c3, cd, ax)) { cleanup(); return vd_set_error(VD_ERR_ARG, "vdt_bottleneck: fused path not eligible"); }
        if ((rc = ctx->make_block(c1, c2, c3, cd, &bi)) || (rc = ctx->add_block(net, bi, ax, aout))) { cleanup(); return rc; }
    } else {
        if ((rc = buf(at1, 64)) || (rc = buf(at2, 64))) { cleanup(); return rc; }
        if ((rc = ctx->add_conv(net, c1, ax, 0, at1, 0)) || (rc = ctx->add_conv(net, c2, at1, 0, at2, 0))) { cleanup(); return rc; }
        if (cd >= 0 && ctx->dual_ok(c3, cd, aout)) {
            rc = ctx->add_conv_dual(net, c3, at2, cd, ax, aout);
        } else if (cd >= 0) {
            if (!(rc = buf(ads, 256)) && !(rc = ctx->add_conv(net, cd, ax, 0, ads, 0)))
                rc = ctx->add_conv(net, c3, at2, 0, aout, 0, &ads, 0, VD_RES_PRE_ACT, 0);
        } else {
            rc = ctx->add_conv(net, c3, at2, 0, aout, 0, &ax, 0, VD_RES_PRE_ACT, 0);
        }
        if (rc) { cleanup(); return rc; }
    }
    rc = ctx->run_ops(net, 0, (int)net.ops.size(), 0, n);
    if (!rc && hipStreamSynchronize(ctx->stream) != hipSuccess) rc = vd_set_error(VD_ERR_HIP, "vdt_bottleneck: sync");
    if (!rc && f32) {
        if (hipMemcpy(y, aout.p, (size_t)n * hh * ww * 256 * 4, hipMemcpyDeviceToHost) != hipSuccess)
            rc = vd_set_error(VD_ERR_HIP, "vdt_bottleneck: download");
    } else if (!rc) {
        std::vector<uint16_t> yb((size_t)n * hh * ww * 256);
        if (hipMemcpy(yb.data(), aout.p, yb.size() * 2, hipMemcpyDeviceToHost) != hipSuccess) {
            rc = vd_set_error(VD_ERR_HIP, "vdt_bottleneck: download");
        } else {
            for (size_t i = 0; i < yb.size(); ++i) {
                const uint32_t u = (uint32_t)yb[i] << 16;
                memcpy(&y[i], &u, 4);
            }
        }
    }
    cleanup();
    return rc;
}
