// runtime.cpp — libvdmi.so: context, weights, network plans and the C-ABI.
//
// Host side of the MI355X detect-and-blur path. One vd_ctx = one GPU + one HIP
// stream + device-resident weights and workspace sized for cfg.max_batch
// frames (replaces the reference's nn.DataParallel replicate-per-forward,
// detect_face/face.py:55-56: weights are uploaded once, workspace is
// allocated once, nothing is allocated on the per-batch path).
#include "../../include/vdmi.h"
#include "vd_common.h"
#include "vd_math.h"
#include "nets.h"

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

static thread_local std::string g_err;

// [a, a + bytes) and [b, b + bytes) share a byte (device frame batches of one geometry)
static bool vd_ranges_overlap(const void* a, const void* b, size_t bytes) {
    const uintptr_t x = (uintptr_t)a, y = (uintptr_t)b;
    return bytes && x < y + bytes && y < x + bytes;
}

int vd_set_error(int code, const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

// ----------------------------------------------------------------------------
// weights container
// ----------------------------------------------------------------------------
int vd_parse_vdw1(const void* blob, size_t bytes, WMap& out) {
    const uint8_t* p = (const uint8_t*)blob;
    const uint8_t* end = p + bytes;
    auto need = [&](size_t k) { return (size_t)(end - p) >= k; };
    if (!need(8) || memcmp(p, "VDW1", 4) != 0) return vd_set_error(VD_ERR_WEIGHTS, "weights: bad magic");
    uint32_t count;
    memcpy(&count, p + 4, 4);
    p += 8;
    for (uint32_t i = 0; i < count; ++i) {
        if (!need(2)) return vd_set_error(VD_ERR_WEIGHTS, "weights: truncated header %u", i);
        uint16_t nl;
        memcpy(&nl, p, 2);
        p += 2;
        if (!need(nl + 2)) return vd_set_error(VD_ERR_WEIGHTS, "weights: truncated name %u", i);
        std::string name((const char*)p, nl);
        p += nl;
        uint8_t dtype = p[0], ndim = p[1];
        p += 2;
        if (dtype != 0 || ndim > 8 || !need(4u * ndim))
            return vd_set_error(VD_ERR_WEIGHTS, "weights: bad tensor header for %s", name.c_str());
        HT t;
        size_t numel = 1;
        for (int d = 0; d < ndim; ++d) {
            uint32_t v;
            memcpy(&v, p, 4);
            p += 4;
            t.shape.push_back((int)v);
            numel *= v;
        }
        if (!need(numel * 4)) return vd_set_error(VD_ERR_WEIGHTS, "weights: truncated data for %s", name.c_str());
        t.data.resize(numel);
        memcpy(t.data.data(), p, numel * 4);
        p += numel * 4;
        out[name] = std::move(t);
    }
    return VD_OK;
}

// ----------------------------------------------------------------------------
// device memory helpers
// ----------------------------------------------------------------------------
int Ctx::dalloc(void** p, size_t bytes) {
    if (bytes == 0) bytes = 16;
    hipError_t e = hipMalloc(p, bytes);
    if (e != hipSuccess) return vd_set_error(VD_ERR_NOMEM, "hipMalloc(%zu) failed: %s", bytes, hipGetErrorString(e));
    allocs.push_back(*p);
    return VD_OK;
}

int Ctx::act(Act& a, int h, int w, int c, bool f32out, bool half) {
    a.h = h; a.w = w; a.c = c;
    a.f32 = !half && (f32out || f32);
    size_t bytes = (size_t)cfg.max_batch * h * w * c * (a.f32 ? 4 : 2);
    int rc = dalloc(&a.p, bytes);
    if (rc) return rc;
    hipMemset(a.p, 0, bytes);
    a.amax = nullptr;
    a.bound = 0.f;
    if (f32 && tune.f32_split == 2) {
        if (!amax_pool && (rc = dalloc((void**)&amax_pool, 2 * amax_region_bytes()))) return rc;
        if (amax_next[amax_owner] >= kAmaxActs) return vd_set_error(VD_ERR_NOMEM, "activation range slots exhausted");
        a.amax = amax_region(amax_owner) + (size_t)amax_next[amax_owner]++ * cfg.max_batch;
    }
    return VD_OK;
}

int Ctx::amax_begin(int owner) {
    amax_owner = owner;
    amax_next[owner] = 0;
    return VD_OK;
}

int Ctx::ensure_pinned(void** p, size_t* have, size_t need) {
    if (*have >= need) return VD_OK;
    if (*p) { (void)hipEventSynchronize(jpeg_ev); hipHostFree(*p); }
    *p = nullptr;
    *have = 0;
    need += need / 4;                             // grow with headroom: batches vary in size
    hipError_t e = hipHostMalloc(p, need, hipHostMallocDefault);
    if (e != hipSuccess) return vd_set_error(VD_ERR_NOMEM, "hipHostMalloc(%zu) failed", need);
    *have = need;
    return VD_OK;
}

int Ctx::ensure_staging(void** p, size_t* have, size_t need) {
    if (*have >= need) return VD_OK;
    if (*p) hipFree(*p);
    *p = nullptr;
    *have = 0;
    hipError_t e = hipMalloc(p, need);
    if (e != hipSuccess) return vd_set_error(VD_ERR_NOMEM, "hipMalloc(%zu) failed", need);
    *have = need;
    return VD_OK;
}

// ----------------------------------------------------------------------------
// conv construction: OIHW f32 -> packed [npad][kpad] in the compute type with
// k = (kh*KW + kw)*cin_pad + c; BN(eval) -> per-channel scale/shift.
// ----------------------------------------------------------------------------
static uint16_t f32_to_bf16_rne(float f) {
    uint32_t u;
    memcpy(&u, &f, 4);
    if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);
    u += 0x7fffu + ((u >> 16) & 1u);
    return (uint16_t)(u >> 16);
}

static uint16_t f32_to_f16_rne(float f) {   // IEEE binary16, round to nearest even (clang _Float16)
    const _Float16 h = (_Float16)f;
    uint16_t u;
    memcpy(&u, &h, 2);
    return u;
}

static float f16_bits_to_f32(uint16_t u) {
    _Float16 h;
    memcpy(&h, &u, 2);
    return (float)h;
}

// host-side 16-bit encoding of the context's half type
static inline uint16_t to_half(bool f16, float v) { return f16 ? f32_to_f16_rne(v) : f32_to_bf16_rne(v); }
static inline float from_half(bool f16, uint16_t u) {
    if (f16) return f16_bits_to_f32(u);
    uint32_t w = (uint32_t)u << 16;
    float v;
    memcpy(&v, &w, 4);
    return v;
}

int Ctx::upload_conv(Conv& cv, const std::vector<float>& w_oihw, const std::vector<float>& scale,
                     const std::vector<float>& shift) {
    const int vec = f32 ? 4 : 8;
    const int bke = 8 * vec;
    cv.cin_pad = (cv.cin + vec - 1) / vec * vec;
    cv.npad = (cv.cout + 127) / 128 * 128;
    const int K = cv.kh * cv.kw * cv.cin_pad;
    cv.kpad = (K + bke - 1) / bke * bke;
    std::vector<float> packed((size_t)cv.npad * cv.kpad, 0.f);
    for (int n = 0; n < cv.cout; ++n)
        for (int c = 0; c < cv.cin; ++c)
            for (int y = 0; y < cv.kh; ++y)
                for (int x = 0; x < cv.kw; ++x)
                    packed[(size_t)n * cv.kpad + (y * cv.kw + x) * cv.cin_pad + c] =
                        w_oihw[(((size_t)n * cv.cin + c) * cv.kh + y) * cv.kw + x];
    int rc;
    if (f32) {
        rc = dalloc(&cv.w, packed.size() * 4);
        if (rc) return rc;
        VD_CHECK_HIP(hipMemcpy(cv.w, packed.data(), packed.size() * 4, hipMemcpyHostToDevice));
        if (tune.f32_split == 2) {   // scaled fp16 pairs (conv_x6.hip, 3 products)
            std::vector<uint16_t> sp(packed.size() * 2);
            std::vector<float> row_inv(cv.npad), sx(cv.npad, 0.f);
            vd_pack_x3h(packed.data(), cv.npad, cv.kpad, sp.data(), row_inv.data());
            for (int n = 0; n < cv.cout; ++n) sx[n] = scale[n] * row_inv[n];
            if ((rc = dalloc(&cv.wx3, sp.size() * 2)) || (rc = dalloc((void**)&cv.scale_x, cv.npad * 4))) return rc;
            VD_CHECK_HIP(hipMemcpy(cv.wx3, sp.data(), sp.size() * 2, hipMemcpyHostToDevice));
            VD_CHECK_HIP(hipMemcpy(cv.scale_x, sx.data(), cv.npad * 4, hipMemcpyHostToDevice));
            cv.split = 2;
        } else if (tune.f32_split) {   // the same weights as three exact bf16 planes for conv_x6.hip
            std::vector<uint16_t> sp(packed.size() * 3);
            vd_pack_x6(packed.data(), cv.npad, cv.kpad, sp.data());
            if ((rc = dalloc(&cv.wx3, sp.size() * 2))) return rc;
            VD_CHECK_HIP(hipMemcpy(cv.wx3, sp.data(), sp.size() * 2, hipMemcpyHostToDevice));
            cv.split = 1;
        }
    } else {
        std::vector<uint16_t> h(packed.size());
        for (size_t i = 0; i < packed.size(); ++i) h[i] = to_half(f16, packed[i]);
        rc = dalloc(&cv.w, h.size() * 2);
        if (rc) return rc;
        VD_CHECK_HIP(hipMemcpy(cv.w, h.data(), h.size() * 2, hipMemcpyHostToDevice));
    }
    std::vector<float> sc(cv.npad, 0.f), sh(cv.npad, 0.f);
    for (int n = 0; n < cv.cout; ++n) { sc[n] = scale[n]; sh[n] = shift[n]; }
    rc = dalloc((void**)&cv.scale, cv.npad * 4);
    if (rc) return rc;
    rc = dalloc((void**)&cv.shift, cv.npad * 4);
    if (rc) return rc;
    VD_CHECK_HIP(hipMemcpy(cv.scale, sc.data(), cv.npad * 4, hipMemcpyHostToDevice));
    VD_CHECK_HIP(hipMemcpy(cv.shift, sh.data(), cv.npad * 4, hipMemcpyHostToDevice));
    cv.flops_per_px = 2.0 * cv.cout * cv.kh * cv.kw * cv.cin;
    return VD_OK;
}

const HT* find_t(const WMap& W, const std::string& k) {
    auto it = W.find(k);
    return it == W.end() ? nullptr : &it->second;
}

// conv weight `wkey` [cout][cin][kh][kw] + BatchNorm at `bn` (eval: alpha =
// gamma/sqrt(var+eps), beta = bias - mean*alpha, as torch's CPU inference kernel).
int Ctx::make_conv_bn(const WMap& W, const std::string& wkey, const std::string& bn, float eps, int stride,
                      int pad, int act, float slope, int* out_idx) {
    return make_conv_bn_cat(W, {{wkey, bn}}, eps, stride, pad, act, slope, out_idx);
}

// Several conv+BN pairs reading the same input, stacked along Cout in the given
// order (the SSH conv5X5_1 + conv3X3 pair of face_net.cpp): one GEMM, per-channel
// scale/shift, so every output channel is computed exactly as by its own conv.
int Ctx::make_conv_bn_cat(const WMap& W, const std::vector<std::pair<std::string, std::string>>& parts, float eps,
                          int stride, int pad, int act, float slope, int* out_idx) {
    Conv cv{};
    std::vector<float> wall, sc, sh;
    for (size_t i = 0; i < parts.size(); ++i) {
        const std::string& wkey = parts[i].first;
        const std::string& bn = parts[i].second;
        const HT* w = find_t(W, wkey);
        if (!w || w->shape.size() != 4) return vd_set_error(VD_ERR_WEIGHTS, "missing/bad conv weight %s", wkey.c_str());
        if (i == 0) { cv.cin = w->shape[1]; cv.kh = w->shape[2]; cv.kw = w->shape[3]; }
        if (w->shape[1] != cv.cin || w->shape[2] != cv.kh || w->shape[3] != cv.kw)
            return vd_set_error(VD_ERR_WEIGHTS, "conv shape mismatch at %s", wkey.c_str());
        const int co = w->shape[0];
        wall.insert(wall.end(), w->data.begin(), w->data.end());
        if (bn.empty()) {
            sc.insert(sc.end(), co, 1.f);
            sh.insert(sh.end(), co, 0.f);
        } else {
            const HT* g = find_t(W, bn + ".weight");
            const HT* b = find_t(W, bn + ".bias");
            const HT* m = find_t(W, bn + ".running_mean");
            const HT* v = find_t(W, bn + ".running_var");
            if (!g || !b || !m || !v) return vd_set_error(VD_ERR_WEIGHTS, "missing BatchNorm tensors under %s", bn.c_str());
            for (int n = 0; n < co; ++n) {
                const float alpha = g->data[n] / std::sqrt(v->data[n] + eps);
                sc.push_back(alpha);
                sh.push_back(b->data[n] - m->data[n] * alpha);
            }
        }
        cv.cout += co;
    }
    cv.stride = stride; cv.pad = pad; cv.act = act; cv.slope = slope;
    int rc = upload_conv(cv, wall, sc, sh);
    if (rc) return rc;
    convs.push_back(cv);
    *out_idx = (int)convs.size() - 1;
    return VD_OK;
}

// Depthwise 3x3 conv [c][1][3][3] + BatchNorm at `bn` (mobilenet025.py:10-14), weights
// stored tap-major [9][c] in the compute type (dwconv.hip reads 16 B of channels per tap).
int Ctx::make_dwconv_bn(const WMap& W, const std::string& wkey, const std::string& bn, float eps, int stride,
                        int act, float slope, int* idx) {
    const HT* w = find_t(W, wkey);
    if (!w || w->shape.size() != 4 || w->shape[1] != 1 || w->shape[2] != 3 || w->shape[3] != 3)
        return vd_set_error(VD_ERR_WEIGHTS, "missing/bad depthwise weight %s", wkey.c_str());
    const HT* g = find_t(W, bn + ".weight");
    const HT* b = find_t(W, bn + ".bias");
    const HT* m = find_t(W, bn + ".running_mean");
    const HT* v = find_t(W, bn + ".running_var");
    if (!g || !b || !m || !v) return vd_set_error(VD_ERR_WEIGHTS, "missing BatchNorm tensors under %s", bn.c_str());
    DwConv d;
    d.c = w->shape[0]; d.stride = stride; d.act = act; d.slope = slope;
    if (d.c % (f32 ? 4 : 8)) return vd_set_error(VD_ERR_WEIGHTS, "depthwise %s: %d channels", wkey.c_str(), d.c);
    std::vector<float> wt((size_t)9 * d.c), sc(d.c), sh(d.c);
    for (int c = 0; c < d.c; ++c) {
        for (int t = 0; t < 9; ++t) wt[(size_t)t * d.c + c] = w->data[(size_t)c * 9 + t];
        const float alpha = g->data[c] / std::sqrt(v->data[c] + eps);
        sc[c] = alpha;
        sh[c] = b->data[c] - m->data[c] * alpha;
    }
    int rc;
    if (f32) {
        if ((rc = dalloc(&d.w, wt.size() * 4))) return rc;
        VD_CHECK_HIP(hipMemcpy(d.w, wt.data(), wt.size() * 4, hipMemcpyHostToDevice));
    } else {
        std::vector<uint16_t> h(wt.size());
        for (size_t i = 0; i < wt.size(); ++i) h[i] = to_half(f16, wt[i]);
        if ((rc = dalloc(&d.w, h.size() * 2))) return rc;
        VD_CHECK_HIP(hipMemcpy(d.w, h.data(), h.size() * 2, hipMemcpyHostToDevice));
    }
    if ((rc = dalloc((void**)&d.scale, d.c * 4)) || (rc = dalloc((void**)&d.shift, d.c * 4))) return rc;
    VD_CHECK_HIP(hipMemcpy(d.scale, sc.data(), d.c * 4, hipMemcpyHostToDevice));
    VD_CHECK_HIP(hipMemcpy(d.shift, sh.data(), d.c * 4, hipMemcpyHostToDevice));
    dwconvs.push_back(d);
    *idx = (int)dwconvs.size() - 1;
    return VD_OK;
}

int Ctx::add_dwconv(Net& net, int di, const Act& x, Act& y) {
    const DwConv& d = dwconvs[di];
    if (x.c < d.c || y.c < d.c || y.h != (x.h - 1) / d.stride + 1 || y.w != (x.w - 1) / d.stride + 1)
        return vd_set_error(VD_ERR_ARG, "depthwise conv plan shape mismatch");
    Op op{};
    op.kind = OP_DWCONV;
    op.conv = di;
    op.x = x;
    op.y = y;
    net.ops.push_back(op);
    return VD_OK;
}

// Several 1x1 conv heads with bias fused along Cout (retinaface.py:90-92,140-142).
// cin_perm (1x1 heads): input channel i of the packed conv reads the tensors' channel
// cin_perm[i] (a concat laid out in another block order)
int Ctx::make_conv_cat(const WMap& W, const std::vector<std::string>& wkeys, const std::vector<std::string>& bkeys,
                       int act, int* out_idx, const std::vector<int>* cin_perm) {
    Conv cv{};
    std::vector<float> wall, sc, sh;
    for (size_t i = 0; i < wkeys.size(); ++i) {
        const HT* w = find_t(W, wkeys[i]);
        const HT* b = bkeys[i].empty() ? nullptr : find_t(W, bkeys[i]);
        if (!w || w->shape.size() != 4 || (!bkeys[i].empty() && !b))
            return vd_set_error(VD_ERR_WEIGHTS, "missing head tensor %s", wkeys[i].c_str());
        if (i == 0) { cv.cin = w->shape[1]; cv.kh = w->shape[2]; cv.kw = w->shape[3]; }
        if (w->shape[1] != cv.cin || w->shape[2] != cv.kh || w->shape[3] != cv.kw)
            return vd_set_error(VD_ERR_WEIGHTS, "head shape mismatch at %s", wkeys[i].c_str());
        wall.insert(wall.end(), w->data.begin(), w->data.end());
        for (int n = 0; n < w->shape[0]; ++n) { sc.push_back(1.f); sh.push_back(b ? b->data[n] : 0.f); }
        cv.cout += w->shape[0];
    }
    if (cin_perm) {
        if ((int)cin_perm->size() != cv.cin || cv.kh != 1 || cv.kw != 1)
            return vd_set_error(VD_ERR_STATE, "internal: head channel permutation");
        std::vector<float> pw(wall.size());
        for (int o = 0; o < cv.cout; ++o)
            for (int i = 0; i < cv.cin; ++i) pw[(size_t)o * cv.cin + i] = wall[(size_t)o * cv.cin + (*cin_perm)[i]];
        wall.swap(pw);
    }
    cv.stride = 1; cv.pad = cv.kh / 2; cv.act = act; cv.slope = 0.f;
    int rc = upload_conv(cv, wall, sc, sh);
    if (rc) return rc;
    convs.push_back(cv);
    *out_idx = (int)convs.size() - 1;
    return VD_OK;
}

// Bottleneck conv3 (ci on x) + downsample (c2 on x2, strided 1x1) in one op.
bool Ctx::dual_ok(int ci, int c2, const Act& y) const {
    const Conv& a = convs[ci];
    const Conv& b = convs[c2];
    if (f32) {   // fp16-pair plan: conv1x1_x6_dual_kernel
        if (!tune.conv_dual || a.split != 2 || b.split != 2 || b.cout != a.cout || b.act != VD_ACT_NONE) return false;
        ConvArgs t{};
        t.kh = a.kh; t.kw = a.kw; t.pad = a.pad; t.stride = a.stride; t.cin_pad = a.cin_pad; t.kpad = a.kpad;
        t.cout = a.cout; t.act = a.act; t.res_mode = VD_RES_NONE; t.ldx = a.cin_pad; t.ldy = y.c;
        t.ldx2 = b.cin_pad; t.cin2_pad = b.cin_pad; t.kpad2 = b.kpad; t.f32_split = 2;
        t.wx3 = a.wx3; t.wx3_2 = b.wx3; t.scale_x = a.scale_x; t.scale2_x = b.scale_x;
        return b.kh == 1 && b.kw == 1 && b.pad == 0 && vd_conv1x1_x6_dual_ok(t);
    }
    ConvArgs t{};
    t.kh = a.kh; t.kw = a.kw; t.pad = a.pad; t.stride = a.stride; t.cin_pad = a.cin_pad; t.kpad = a.kpad;
    t.cout = a.cout; t.act = a.act; t.res_mode = VD_RES_NONE; t.ldx = a.cin_pad; t.ldy = y.c; t.x2 = (const void*)1;
    t.cin2_pad = b.cin_pad; t.kpad2 = b.kpad; t.ldx2 = b.cin_pad; t.tune = &tune;
    return b.kh == 1 && b.kw == 1 && b.pad == 0 && b.cout == a.cout && b.act == VD_ACT_NONE && vd_conv1x1_dual_ok(t);
}

int Ctx::add_conv_dual(Net& net, int ci, const Act& x, int c2, const Act& x2, Act& y) {
    int rc = add_conv(net, ci, x, 0, y, 0);
    if (rc) return rc;
    const Conv& b = convs[c2];
    if ((x2.h - 1) / b.stride + 1 != y.h || (x2.w - 1) / b.stride + 1 != y.w || b.cin_pad > x2.c)
        return vd_set_error(VD_ERR_ARG, "dual conv plan shape mismatch");
    net.ops.back().conv2 = c2;
    net.ops.back().x2 = x2;
    return VD_OK;
}

int Ctx::add_conv(Net& net, int ci, const Act& x, int xcoff, Act& y, int ycoff, const Act* res, int rcoff, int rmode,
                  int rup) {
    const Conv& cv = convs[ci];
    Op op{};
    op.kind = OP_CONV;
    op.conv = ci;
    op.x = x; op.xcoff = xcoff;
    op.y = y; op.ycoff = ycoff;
    if (res) { op.r = *res; op.rcoff = rcoff; op.rmode = rmode; op.rup = rup; }
    const int oh = (x.h + 2 * cv.pad - cv.kh) / cv.stride + 1;
    const int ow = (x.w + 2 * cv.pad - cv.kw) / cv.stride + 1;
    const int xspan = cv.grp_co ? (cv.cout / cv.grp_co - 1) * cv.grp_ci + cv.cin_pad : cv.cin_pad;
    if (oh != y.h || ow != y.w || ycoff + cv.cout > y.c || xcoff + xspan > x.c)
        return vd_set_error(VD_ERR_ARG, "conv plan shape mismatch (%dx%d vs %dx%d)", oh, ow, y.h, y.w);
    net.ops.push_back(op);
    return VD_OK;
}

// ----------------------------------------------------------------------------
// plan execution
// ----------------------------------------------------------------------------
void Ctx::t_begin(int fam, double work) {
    if (!timing) return;
    if (ev_used == ev_pool.size()) {
        TimedEv t{};
        hipEventCreate(&t.a);
        hipEventCreate(&t.b);
        ev_pool.push_back(t);
    }
    TimedEv& t = ev_pool[ev_used];
    t.fam = fam;
    t.work = work;
    hipEventRecord(t.a, stream);
}

void Ctx::t_end() {
    if (!timing) return;
    hipEventRecord(ev_pool[ev_used].b, stream);
    ++ev_used;
}

static inline const void* foff(const Act& a, int f0) {
    return a.p ? (const char*)a.p + (size_t)f0 * a.h * a.w * a.c * (a.f32 ? 4 : 2) : nullptr;
}

int Ctx::run_conv_op(const Op& op, int f0, int n, int fam) {
    const Conv& cv = convs[op.conv];
    ConvArgs a{};
    a.x = foff(op.x, f0); a.xh = op.x.h; a.xw = op.x.w; a.ldx = op.x.c; a.xcoff = op.xcoff;
    a.w = cv.w; a.scale = cv.scale; a.shift = cv.shift;
    a.res = foff(op.r, f0); a.res_ld = op.r.c; a.res_coff = op.rcoff; a.res_up = op.rup; a.rh = op.r.h; a.rw = op.r.w;
    a.res_mode = op.r.p ? op.rmode : VD_RES_NONE;
    a.y = (void*)foff(op.y, f0); a.yh = op.y.h; a.yw = op.y.w; a.ldy = op.y.c; a.ycoff = op.ycoff;
    a.B = n; a.cin_pad = cv.cin_pad; a.cout = cv.cout; a.kpad = cv.kpad;
    a.kh = cv.kh; a.kw = cv.kw; a.stride = cv.stride; a.pad = cv.pad;
    a.M = n * op.y.h * op.y.w;
    a.act = cv.act; a.slope = cv.slope; a.out_f32 = op.y.f32 ? 1 : 0;
    a.f16 = f16 ? 1 : 0;
    a.tune = &tune;
    a.wx3 = cv.wx3;
    a.scale_x = cv.scale_x;
    a.f32_split = cv.split;
    a.xmax = op.x.amax ? op.x.amax + f0 : nullptr;
    a.xbound = op.x.bound;
    a.x_exact = (op.x.exact16 && cv.split == 2 && tune.x6_exact) ? 1 : 0;
    a.ymax = op.y.amax ? op.y.amax + f0 : nullptr;
    a.grp_co = cv.grp_co; a.grp_ci = cv.grp_ci;
    if (cv.split == 2 && !a.xmax && !(a.xbound > 0.f))
        return vd_set_error(VD_ERR_ARG, "internal: conv input without a range (fp16-pair plan)");
    if (a.xmax && op.x.amax == op.y.amax) {
        // input and output are channel slices of one buffer (the SSH concat): the kernel
        // reads the input's per-frame range while its epilogue raises the same slots, so
        // it reads a copy frozen before the launch (one array per conv: the frame groups
        // run the same conv concurrently on disjoint frames)
        unsigned*& snap = amax_snaps[op.conv];
        if (!snap) {
            int rc = dalloc((void**)&snap, (size_t)cfg.max_batch * 4);
            if (rc) return rc;
        }
        VD_CHECK_HIP(hipMemcpyAsync(snap + f0, a.xmax, (size_t)n * 4, hipMemcpyDeviceToDevice, stream));
        a.xmax = snap + f0;
    }
    double flops = cv.flops_per_px * a.M;
    if (op.conv2 >= 0) {
        const Conv& c2 = convs[op.conv2];
        a.x2 = foff(op.x2, f0); a.xh2 = op.x2.h; a.xw2 = op.x2.w; a.ldx2 = op.x2.c; a.xcoff2 = 0;
        a.stride2 = c2.stride; a.w2 = c2.w; a.scale2 = c2.scale; a.shift2 = c2.shift;
        a.cin2_pad = c2.cin_pad; a.kpad2 = c2.kpad;
        a.wx3_2 = c2.wx3; a.scale2_x = c2.scale_x;
        a.x2max = op.x2.amax ? op.x2.amax + f0 : nullptr;
        a.x2bound = op.x2.bound;
        flops += c2.flops_per_px * a.M;
    }
    t_begin(fam, flops);
    hipError_t e = vd_launch_conv(a, f32, stream);
    t_end();
    if (e != hipSuccess) return vd_set_error(VD_ERR_HIP, "conv launch: %s", hipGetErrorString(e));
    return VD_OK;
}

// conv3 (+ identity) of one bottleneck and conv1 of the next in one pass (chain.hip)
int Ctx::run_chain_op(const Op& op, int f0, int n, int fam) {
    const Conv& c3 = convs[op.conv];
    const Conv& c1 = convs[op.conv2];
    if (f32) {   // fp16-pair plan (chain32.hip)
        Chain32Args a{};
        a.t2 = foff(op.x, f0); a.ld_t2 = op.x.c;
        a.res = foff(op.r, f0); a.ld_res = op.r.c;
        a.w3 = c3.wx3; a.w1 = c1.wx3_chain;
        a.sc3 = c3.scale_x; a.sh3 = c3.shift; a.sc1 = c1.scale_x; a.sh1 = c1.shift;
        a.y = (void*)foff(op.y, f0); a.ld_y = op.y.c;
        a.y2 = (void*)foff(op.y2, f0); a.ld_y2 = op.y2.c;
        a.hw = op.y.h * op.y.w;
        a.M = n * a.hw;
        a.B = n;
        a.xmax = op.x.amax ? op.x.amax + f0 : nullptr; a.xbound = op.x.bound;
        a.ymax = op.y.amax ? op.y.amax + f0 : nullptr;
        a.y2max = op.y2.amax ? op.y2.amax + f0 : nullptr;
        a.gpw = tune.chain_gpw;
        t_begin(fam, (c3.flops_per_px + c1.flops_per_px) * a.M);
        hipError_t e = vd_launch_chain32(a, stream);
        t_end();
        if (e != hipSuccess) return vd_set_error(VD_ERR_HIP, "chain32 launch: %s", hipGetErrorString(e));
        return VD_OK;
    }
    ChainArgs a{};
    a.t2 = foff(op.x, f0); a.ld_t2 = op.x.c;
    a.res = foff(op.r, f0); a.ld_res = op.r.c;
    a.w3 = c3.w; a.kpad3 = c3.kpad; a.sc3 = c3.scale; a.sh3 = c3.shift;
    a.w1 = c1.w; a.kpad1 = c1.kpad; a.sc1 = c1.scale; a.sh1 = c1.shift;
    a.y = (void*)foff(op.y, f0); a.ld_y = op.y.c;
    a.y2 = (void*)foff(op.y2, f0); a.ld_y2 = op.y2.c;
    a.M = n * op.y.h * op.y.w;
    a.f16 = f16 ? 1 : 0;
    t_begin(fam, (c3.flops_per_px + c1.flops_per_px) * a.M);
    hipError_t e = vd_launch_chain(a, stream);
    t_end();
    if (e != hipSuccess) return vd_set_error(VD_ERR_HIP, "chain launch: %s", hipGetErrorString(e));
    return VD_OK;
}

// Peephole over ops [begin, end) of a bf16 / fp16 plan: a bottleneck conv3 (1x1, + identity
// before the ReLU) immediately followed by a 1x1 conv that reads exactly its output
// (the next bottleneck's conv1) becomes one OP_CHAIN where chain.hip covers the shape.
// fp32 plan (chain32.hip): the same peephole on the layer2 shape with fp16-pair weights;
// conv1's planes are copied with K permuted inside each 32-channel step (position 8q + e
// <- channel 4q + e, 8q + 4 + e <- 16 + 4q + e) so conv3's accumulator lanes are its B
// fragments.
int Ctx::chain32_weights(Conv& c1) {
    if (c1.wx3_chain) return VD_OK;
    const size_t rows = (size_t)c1.npad, nk = (size_t)c1.kpad / 32, bytes = rows * nk * 2 * 64;
    std::vector<uint16_t> src(bytes / 2), dst(bytes / 2);
    VD_CHECK_HIP(hipMemcpy(src.data(), c1.wx3, bytes, hipMemcpyDeviceToHost));
    for (size_t blk = 0; blk < rows * nk * 2; ++blk)       // one 32-entry plane of one k-step of one row
        for (int qq = 0; qq < 4; ++qq)
            for (int e = 0; e < 4; ++e) {
                dst[blk * 32 + 8 * qq + e] = src[blk * 32 + 4 * qq + e];
                dst[blk * 32 + 8 * qq + 4 + e] = src[blk * 32 + 16 + 4 * qq + e];
            }
    int rc = dalloc(&c1.wx3_chain, bytes);
    if (rc) return rc;
    VD_CHECK_HIP(hipMemcpy(c1.wx3_chain, dst.data(), bytes, hipMemcpyHostToDevice));
    return VD_OK;
}

void Ctx::fuse_chains(Net& net, size_t begin) {
    if (f32) {
        fuse_chains32(net, begin);
        return;
    }
    std::vector<Op> out(net.ops.begin(), net.ops.begin() + begin);
    for (size_t i = begin; i < net.ops.size(); ++i) {
        const Op& a = net.ops[i];
        if (i + 1 < net.ops.size() && a.kind == OP_CONV && net.ops[i + 1].kind == OP_CONV && a.conv2 < 0) {
            const Op& b = net.ops[i + 1];
            const Conv& c3 = convs[a.conv];
            const Conv& c1 = convs[b.conv];
            const bool shape = c3.kh == 1 && c3.kw == 1 && c3.stride == 1 && c3.pad == 0 && c3.act == VD_ACT_RELU &&
                               c1.kh == 1 && c1.kw == 1 && c1.stride == 1 && c1.pad == 0 && c1.act == VD_ACT_RELU &&
                               a.r.p && a.rmode == VD_RES_PRE_ACT && !a.rup && a.rcoff == 0 && a.xcoff == 0 &&
                               a.ycoff == 0 && b.conv2 < 0 && !b.r.p && b.x.p == a.y.p && b.xcoff == 0 &&
                               b.ycoff == 0 && !a.y.f32 && !b.y.f32 && c3.cin_pad == a.x.c &&
                               c1.cin_pad == c3.cout && a.r.h == a.y.h && a.r.w == a.y.w;
            const long M = (long)cfg.max_batch * a.y.h * a.y.w;
            if (shape && tune.chain && vd_chain_ok(c3.cin_pad, c3.cout, c3.kpad, c1.kpad, a.x.c, a.r.c, a.y.c, b.y.c, M)) {
                Op op = a;
                op.kind = OP_CHAIN;
                op.conv2 = b.conv;
                op.y2 = b.y;
                out.push_back(op);
                ++i;
                continue;
            }
        }
        out.push_back(a);
    }
    net.ops.swap(out);
}

void Ctx::fuse_chains32(Net& net, size_t begin) {
    if (!tune.chain) return;
    std::vector<Op> out(net.ops.begin(), net.ops.begin() + begin);
    for (size_t i = begin; i < net.ops.size(); ++i) {
        const Op& a = net.ops[i];
        if (i + 1 < net.ops.size() && a.kind == OP_CONV && net.ops[i + 1].kind == OP_CONV && a.conv2 < 0) {
            const Op& b = net.ops[i + 1];
            const Conv& c3 = convs[a.conv];
            Conv& c1 = convs[b.conv];
            const bool shape = c3.kh == 1 && c3.kw == 1 && c3.stride == 1 && c3.pad == 0 && c3.act == VD_ACT_RELU &&
                               c1.kh == 1 && c1.kw == 1 && c1.stride == 1 && c1.pad == 0 && c1.act == VD_ACT_RELU &&
                               c3.split == 2 && c1.split == 2 && c3.wx3 && c1.wx3 && c3.scale_x && c1.scale_x &&
                               a.r.p && a.rmode == VD_RES_PRE_ACT && !a.rup && a.rcoff == 0 && a.xcoff == 0 &&
                               a.ycoff == 0 && b.conv2 < 0 && !b.r.p && b.x.p == a.y.p && b.xcoff == 0 &&
                               b.ycoff == 0 && a.x.f32 && a.y.f32 && b.y.f32 && a.r.f32 && c3.cin_pad == a.x.c &&
                               c1.cin_pad == c3.cout && a.r.h == a.y.h && a.r.w == a.y.w;
            const long M = (long)cfg.max_batch * a.y.h * a.y.w;
            const bool take = tune.chain == 1 || c3.cin_pad == 128;   // option chain=2 (default): layer2 only
            if (shape && take && vd_chain32_ok(c3.cin_pad, c3.cout, c3.kpad, c1.kpad, a.x.c, a.r.c, a.y.c, b.y.c, M,
                                       cfg.max_batch) &&
                chain32_weights(c1) == VD_OK) {
                Op op = a;
                op.kind = OP_CHAIN;
                op.conv2 = b.conv;
                op.y2 = b.y;
                out.push_back(op);
                ++i;
                continue;
            }
        }
        out.push_back(a);
    }
    net.ops.swap(out);
}

int Ctx::run_dwconv_op(const Op& op, int f0, int n) {
    const DwConv& d = dwconvs[op.conv];
    DwConvArgs a{};
    a.x = foff(op.x, f0); a.xh = op.x.h; a.xw = op.x.w; a.ldx = op.x.c; a.xcoff = 0;
    a.w = d.w; a.scale = d.scale; a.shift = d.shift;
    a.y = (void*)foff(op.y, f0); a.yh = op.y.h; a.yw = op.y.w; a.ldy = op.y.c; a.ycoff = 0;
    a.B = n; a.c = d.c; a.stride = d.stride; a.act = d.act; a.slope = d.slope;
    a.ymax = op.y.amax ? op.y.amax + f0 : nullptr;
    t_begin(4, 0);
    hipError_t e = vd_launch_dwconv(a, f32, f16, stream);
    t_end();
    if (e != hipSuccess) return vd_set_error(VD_ERR_HIP, "depthwise conv: %s", hipGetErrorString(e));
    return VD_OK;
}

// max-pool / upsample: the output's per-frame range is within the input's
static hipError_t amax_follow_impl(const Op& op, int f0, int n, hipStream_t s) {
    if (!op.y.amax || op.y.amax == op.x.amax) return hipSuccess;   // in-place slices: already covered
    if (!op.x.amax) return op.x.bound > 0.f ? hipErrorInvalidValue : hipSuccess;
    return vd_launch_amax_merge(op.y.amax + f0, op.x.amax + f0, n, s);
}

int Ctx::run_ops(const Net& net, int b, int e, int f0, int n) {
    // two lanes (face net, option ssh_side): lane-1 ops run on stream_side; an op with
    // dep >= 0 waits for that op's completion event first (recorded below on the
    // producer's lane); after the net's last op the main lane waits for the side lane
    const bool lanes = &net == &face.net && !lane_ev.empty();
    hipStream_t main = stream;
    bool side_used = false;
    for (int i = b; i < e; ++i) {
        const Op& op = net.ops[i];
        int rc = VD_OK;
        if (lanes) {
            stream = op.lane ? stream_side : main;
            side_used |= op.lane != 0;
            if (op.dep >= 0) VD_CHECK_HIP(hipStreamWaitEvent(stream, lane_ev[op.dep], 0));
        }
        if (op.kind == OP_CONV) {
            rc = run_conv_op(op, f0, n, net.conv_fam);
        } else if (op.kind == OP_BLOCK) {
            rc = run_block_op(op, f0, n, net.conv_fam);
        } else if (op.kind == OP_CHAIN) {
            rc = run_chain_op(op, f0, n, net.conv_fam);
        } else if (op.kind == OP_STEMPOOL) {
            rc = run_stem_pool_op(op, f0, n, net.conv_fam);
        } else if (op.kind == OP_DWCONV) {
            rc = run_dwconv_op(op, f0, n);
        } else if (op.kind == OP_MAXPOOL) {
            t_begin(4, 0);
            hipError_t er = vd_launch_maxpool(f32, f16, foff(op.x, f0), n, op.x.h, op.x.w, op.x.c, op.xcoff,
                                              (void*)foff(op.y, f0), op.y.h, op.y.w, op.y.c, op.ycoff, op.ch, op.k,
                                              op.s, op.p, stream);
            t_end();
            if (er == hipSuccess) er = amax_follow_impl(op, f0, n, stream);
            if (er != hipSuccess) rc = vd_set_error(VD_ERR_HIP, "maxpool: %s", hipGetErrorString(er));
        } else if (op.kind == OP_UPSAMPLE) {
            t_begin(4, 0);
            hipError_t er = vd_launch_upsample2x(f32, foff(op.x, f0), n, op.x.h, op.x.w, op.x.c, op.xcoff,
                                                 (void*)foff(op.y, f0), op.y.c, op.ycoff, op.ch, stream);
            t_end();
            if (er == hipSuccess) er = amax_follow_impl(op, f0, n, stream);
            if (er != hipSuccess) rc = vd_set_error(VD_ERR_HIP, "upsample: %s", hipGetErrorString(er));
        }
        if (lanes && lane_ev[i]) VD_CHECK_HIP(hipEventRecord(lane_ev[i], stream));
        if (lanes) stream = main;
        if (rc) return rc;
        if (&net == &face.net && i + 1 == fork_at) VD_CHECK_HIP(hipEventRecord(ev_fork, stream));
    }
    if (lanes && side_used) {
        VD_CHECK_HIP(hipEventRecord(ev_side, stream_side));
        VD_CHECK_HIP(hipStreamWaitEvent(stream, ev_side, 0));
    }
    return VD_OK;
}

// The face net's op list as built (FPN o3 o2 m2 o1 m1, then SSH + heads of levels 0, 1,
// 2) reordered into two lanes: level 2's chain right after o3 and level 1's after m2,
// both on the side stream, so they fill the CUs that FPN merge1 and the level-0 SSH
// convs (6x the pixels) leave idle in their last partial rounds. Same kernels and
// operands: results are bit-identical to the one-lane order.
int Ctx::face_lanes(const int (&fpn)[5], const int (&ssh_b)[3], const int (&ssh_e)[3]) {
    Net& net = face.net;
    std::vector<Op> out(net.ops.begin(), net.ops.begin() + fpn[0]);
    auto take = [&](int b, int e, int lane, int dep) {
        for (int i = b; i < e; ++i) {
            Op op = net.ops[i];
            op.lane = lane;
            op.dep = i == b ? dep : -1;
            out.push_back(op);
        }
    };
    take(fpn[0], fpn[0] + 1, 0, -1);                      // o3
    const int p_o3 = (int)out.size() - 1;
    take(ssh_b[2], ssh_e[2], 1, p_o3);                     // level 2 (reads o3)
    take(fpn[1], fpn[2] + 1, 0, -1);                       // o2, m2
    const int p_m2 = (int)out.size() - 1;
    take(ssh_b[1], ssh_e[1], 1, p_m2);                     // level 1 (reads m2)
    take(fpn[3], fpn[4] + 1, 0, -1);                       // o1, m1
    take(ssh_b[0], ssh_e[0], 0, -1);                       // level 0
    if (out.size() != net.ops.size()) return vd_set_error(VD_ERR_STATE, "internal: face lanes lost ops");
    net.ops.swap(out);
    if (!stream_side) {
        VD_CHECK_HIP(hipStreamCreateWithFlags(&stream_side, hipStreamNonBlocking));
        VD_CHECK_HIP(hipEventCreateWithFlags(&ev_side, hipEventDisableTiming));
    }
    for (hipEvent_t ev : lane_ev)
        if (ev) hipEventDestroy(ev);
    lane_ev.assign(net.ops.size(), nullptr);
    for (int i : {p_o3, p_m2}) VD_CHECK_HIP(hipEventCreateWithFlags(&lane_ev[i], hipEventDisableTiming));
    return VD_OK;
}

// Depth-first over micro-batches of `mb` frames for ops [0, split) -- each
// micro-batch's stem/layer1/layer2 intermediates (~100-200 MB) then stay in the
// 256 MiB Infinity Cache between producer and consumer -- then ops [split, end)
// over the whole batch (the small late layers need the whole batch to fill 256 CUs).
int Ctx::run_net(const Net& net, int n, int mb, int split) {
    const int ne = (int)net.ops.size();
    if (net.amax) VD_CHECK_HIP(hipMemsetAsync(net.amax, 0, net.amax_bytes, stream));
    if (mb <= 0 || mb >= n || split <= 0) return run_ops(net, 0, ne, 0, n);
    for (int f0 = 0; f0 < n; f0 += mb) {
        int rc = run_ops(net, 0, split, f0, std::min(mb, n - f0));
        if (rc) return rc;
    }
    return run_ops(net, split, ne, 0, n);
}

// cv2.resize mode selection (resize.cpp hal::resize [ext]; oracle/letterbox.py)
void vd_resize_mode(int ih, int iw, int nh, int nw, int* mode, double* sx, double* sy) {
    if (nh == ih && nw == iw) { *mode = LB_COPY; *sx = *sy = 1.0; return; }
    double inv_x = (double)nw / iw, inv_y = (double)nh / ih;
    double scx = 1.0 / inv_x, scy = 1.0 / inv_y;
    int isx = (int)std::nearbyint(scx), isy = (int)std::nearbyint(scy);
    bool area_fast = std::fabs(scx - isx) < 2.220446049250313e-16 && std::fabs(scy - isy) < 2.220446049250313e-16;
    *mode = (area_fast && isx == 2 && isy == 2) ? LB_AREA2 : LB_LINEAR;
    *sx = scx;
    *sy = scy;
}

const uint8_t* Ctx::frames_to_device(const uint8_t* frames, int n, int h, size_t pitch, int where, int* rc) {
    *rc = VD_OK;
    if (where == VD_DEVICE) return frames;
    size_t bytes = (size_t)n * h * pitch;
    *rc = ensure_staging(&stage_in, &stage_in_bytes, bytes);
    if (*rc) return nullptr;
    hipError_t e = hipMemcpyAsync(stage_in, frames, bytes, hipMemcpyHostToDevice, stream);
    if (e != hipSuccess) {
        *rc = vd_set_error(VD_ERR_HIP, "H2D frames: %s", hipGetErrorString(e));
        return nullptr;
    }
    return (const uint8_t*)stage_in;
}

int Ctx::check_frames(int n, int h, int w, size_t pitch) {
    if (n <= 0 || n > cfg.max_batch) return vd_set_error(VD_ERR_ARG, "n=%d outside [1, max_batch=%d]", n, cfg.max_batch);
    if (h <= 0 || w <= 0 || pitch < (size_t)w * 3) return vd_set_error(VD_ERR_ARG, "bad frame geometry %dx%d pitch %zu", w, h, pitch);
    return VD_OK;
}

// Box outputs: kernels write straight into caller arrays when they are device
// memory; host outputs go through ctx staging + one D2H at the end. `out` may be
// NULL (no caller copy; the complete lists stay readable through vd_read_boxes).
int Ctx::box_targets(vd_boxes* out, int n, BoxTargets& t) {
    t = BoxTargets{};
    if (!out) return VD_OK;
    if (!out->count || !out->xyxy || out->cap <= 0) return vd_set_error(VD_ERR_ARG, "vd_boxes needs count, xyxy, cap>0");
    t.cap = out->cap;
    if (out->where == VD_DEVICE) {
        t.count = out->count; t.xyxy = out->xyxy; t.xyxy_f = out->xyxy_f; t.score = out->score; t.label = out->label;
        return VD_OK;
    }
    return host_box_staging(&stage_box, &stage_box_bytes, out->cap, n, t);
}

int Ctx::host_box_staging(void** buf, size_t* have, int cap, int n, BoxTargets& t) {
    size_t nb = (size_t)n * cap;
    size_t need = n * 4 + nb * (16 + 16 + 4 + 4);
    int rc = ensure_staging(buf, have, need + 64);
    if (rc) return rc;
    char* p = (char*)*buf;
    t.cap = cap;
    t.count = (int*)p; p += ((n * 4 + 15) / 16) * 16;
    t.xyxy = (int*)p; p += nb * 16;
    t.xyxy_f = (float*)p; p += nb * 16;
    t.score = (float*)p; p += nb * 4;
    t.label = (int*)p;
    return VD_OK;
}

// Host outputs: one D2H of the staged arrays. count[f] is the complete keep count,
// which may exceed cap: the arrays then hold the first cap boxes, the rest stay
// readable through vd_read_boxes, and the mosaic used every box regardless.
int Ctx::box_finish(vd_boxes* out, int n, const BoxTargets& t) {
    if (!out || out->where == VD_DEVICE) return VD_OK;
    size_t nb = (size_t)n * out->cap;
    VD_CHECK_HIP(hipMemcpyAsync(out->count, t.count, n * 4, hipMemcpyDeviceToHost, stream));
    VD_CHECK_HIP(hipMemcpyAsync(out->xyxy, t.xyxy, nb * 16, hipMemcpyDeviceToHost, stream));
    if (out->xyxy_f) VD_CHECK_HIP(hipMemcpyAsync(out->xyxy_f, t.xyxy_f, nb * 16, hipMemcpyDeviceToHost, stream));
    if (out->score) VD_CHECK_HIP(hipMemcpyAsync(out->score, t.score, nb * 4, hipMemcpyDeviceToHost, stream));
    if (out->label) VD_CHECK_HIP(hipMemcpyAsync(out->label, t.label, nb * 4, hipMemcpyDeviceToHost, stream));
    VD_CHECK_HIP(hipStreamSynchronize(stream));
    return VD_OK;
}

int Ctx::face_letterbox(const uint8_t* dframes, int n, int h, int w, size_t pitch) {
    LetterboxArgs a;
    face_letterbox_args(dframes, n, h, w, pitch, &a);
    t_begin(2, (double)n * (a.nh * (double)w * 3 + (double)a.oh * a.ow * a.cpad * (f32 ? 4 : 2)));
    hipError_t e = vd_launch_letterbox(a, stream);
    t_end();
    if (e != hipSuccess) return vd_set_error(VD_ERR_HIP, "letterbox: %s", hipGetErrorString(e));
    return VD_OK;
}

void Ctx::face_letterbox_args(const uint8_t* dframes, int n, int h, int w, size_t pitch, LetterboxArgs* out) {
    LetterboxArgs a{};
    a.src = dframes; a.n = n; a.ih = h; a.iw = w; a.pitch = pitch;
    a.oh = face.in_h; a.ow = face.in_w;
    // utils/utils.py:9-13 (Python doubles)
    double scale = std::min((double)a.ow / w, (double)a.oh / h);
    a.nw = (int)(w * scale);
    a.nh = (int)(h * scale);
    a.top = (a.oh - a.nh) / 2;
    a.left = (a.ow - a.nw) / 2;
    vd_resize_mode(h, w, a.nh, a.nw, &a.mode, &a.scale_x, &a.scale_y);
    a.pad_value = 128.f;
    a.mean[0] = 104.f; a.mean[1] = 117.f; a.mean[2] = 123.f;
    a.div = 1.f;
    a.flip = 0;
    // fp32 plan with the fused stem: an fp16 space-to-depth canvas (integer values, exact)
    a.out = face.input.p; a.cpad = face.input.c; a.out_f32 = face.input.f32 ? 1 : 0;
    a.out_f16 = (f16 || (f32 && !face.input.f32)) ? 1 : 0;
    a.s2d = face.s2d ? 1 : 0;
    *out = a;
}

int Ctx::face_forward(int n) {
    const int mb = cfg.reserved[0];                       // frames per micro-batch (0 = off)
    const int stage = cfg.reserved[1] > 0 ? cfg.reserved[1] : 2;   // micro-batch through layer<stage>
    const int split = face.net.stage_end[std::min(std::max(stage, 0), 4)];
    const int G = std::min(std::min(tune.face_groups, 4), n);
    if (G >= 2 && mb <= 0 && lane_ev.empty()) {
        // G frame groups on G streams (group 0 on the context stream): each layer's last
        // partial round of workgroups leaves CUs that the other groups' launches take.
        // Every kernel is batch-invariant (a frame's sums do not depend on its batch
        // position or the launch's frame count), so the results are bit-identical to
        // one launch over n frames.
        const Net& net = face.net;
        while ((int)group_streams.size() < G - 1) {
            hipStream_t st;
            hipEvent_t ev;
            VD_CHECK_HIP(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
            VD_CHECK_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
            group_streams.push_back(st);
            group_events.push_back(ev);
        }
        if (!ev_half) VD_CHECK_HIP(hipEventCreateWithFlags(&ev_half, hipEventDisableTiming));
        if (net.amax) VD_CHECK_HIP(hipMemsetAsync(net.amax, 0, net.amax_bytes, stream));
        VD_CHECK_HIP(hipEventRecord(ev_half, stream));
        const int ne = (int)net.ops.size();
        hipStream_t main = stream;
        for (int g = 0; g < G; ++g) {
            const int f0 = (int)((long)n * g / G), f1 = (int)((long)n * (g + 1) / G);
            stream = g ? group_streams[g - 1] : main;
            if (g) VD_CHECK_HIP(hipStreamWaitEvent(stream, ev_half, 0));
            int rc = run_ops(net, 0, ne, f0, f1 - f0);
            if (!rc && g && hipEventRecord(group_events[g - 1], stream) != hipSuccess)
                rc = vd_set_error(VD_ERR_HIP, "group event");
            stream = main;
            if (rc) return rc;
        }
        for (int g = 1; g < G; ++g) VD_CHECK_HIP(hipStreamWaitEvent(stream, group_events[g - 1], 0));
        return VD_OK;
    }
    return run_net(face.net, n, mb, split);
}

int Ctx::face_post(int n, int img_h, int img_w, const BoxTargets& t) {
    PostArgs p{};
    p.mode = POST_FACE;
    for (int l = 0; l < 3; ++l) {
        p.heads[l] = (const float*)face.heads[l].p;
        p.lh[l] = face.heads[l].h;
        p.lw[l] = face.heads[l].w;
        p.loff[l] = face.loff[l];
    }
    p.hstride = face.heads[0].c;
    p.anchors = face.anchors; p.A = face.A; p.B = n;
    p.conf = cfg.confidence; p.iou = cfg.nms_iou; p.max_det = 0;
    p.cand_keys = face.post.keys; p.cand_count = face.post.count;
    p.scratch_box = face.post.box; p.scratch_cls = face.post.cls; p.scratch_nbox = face.post.nbox;
    p.scratch_area = face.post.area; p.scratch_keys = face.post.sort; p.scratch_supp = face.post.supp;
    p.sort_cap = face.post.sort_cap;
    p.img_h = img_h; p.img_w = img_w;
    // retinaface_correct_boxes factors (utils_bbox.py:118-132), float32 tensor arithmetic
    const float inh = (float)face.in_h, inw = (float)face.in_w, ih = (float)img_h, iw = (float)img_w;
    const float rh = inh / ih, rw = inw / iw;
    const float mn = rh < rw ? rh : rw;
    const float nh = ih * mn, nw = iw * mn;
    p.offy = ((inh - nh) / 2.0f) / inh;
    p.offx = ((inw - nw) / 2.0f) / inw;
    p.scy = inh / nh;
    p.scx = inw / nw;
    p.cap = t.cap; p.out_count = t.count; p.out_xyxy = t.xyxy; p.out_xyxy_f = t.xyxy_f;
    p.out_score = t.score; p.out_label = t.label;
    vd_post_keep_args(face.post, p, n);
    t_begin(3, (double)n * face.A * 32 * 4);
    hipError_t e = vd_launch_post(p, stream);
    t_end();
    if (e != hipSuccess) return vd_set_error(VD_ERR_HIP, "face post: %s", hipGetErrorString(e));
    return VD_OK;
}

int Ctx::launch_mosaic(const uint8_t* in, uint8_t* out, int n, int h, int w, size_t pitch, const int* cnt0,
                       const int* xy0, int cap0, const int* cnt1, const int* xy1, int cap1, int level) {
    const int tcap = (cnt0 ? cap0 : 0) + (cnt1 ? cap1 : 0);
    int rc = ensure_staging(&mosaic_table, &mosaic_table_bytes, vd_mosaic_table_bytes(n, tcap) + 64);
    if (rc) return rc;
    const int map_on = tune.mosaic_map | (tune.mosaic_nt << 1) | (tune.mosaic_gather ? 16 : 0) | ((tune.mosaic_rows & 63) << 8);
    auto launch = [&](int stages) {
        return vd_launch_mosaic(in, out, n, h, w, pitch, cnt0, xy0, cap0, cnt1, xy1, cap1, level, mosaic_table, stages,
                                map_on, tune.mosaic_cells, stream);
    };
    hipError_t e = hipSuccess;
    if (tune.mosaic_fused) {
        // one launch: the output pass walks and gathers its bands' cells itself (family 1)
        t_begin(1, 2.0 * n * (double)h * w * 3);
        e = launch(8);
        t_end();
    } else {
        t_begin(6, 0);
        e = launch(1);
        t_end();
        if (e == hipSuccess) {
            t_begin(1, 2.0 * n * (double)h * w * 3);
            e = launch(2);
            t_end();
        }
    }
    if (e != hipSuccess) return vd_set_error(VD_ERR_HIP, "mosaic: %s", hipGetErrorString(e));
    return VD_OK;
}

// ----------------------------------------------------------------------------
// C-ABI
// ----------------------------------------------------------------------------
#define VD_ENTRY(ctx)                                                          \
    if (!(ctx)) return vd_set_error(VD_ERR_ARG, "null context");              \
    std::lock_guard<std::mutex> _lk((ctx)->mu);                                \
    if (hipSetDevice((ctx)->device) != hipSuccess)                             \
        return vd_set_error(VD_ERR_HIP, "hipSetDevice(%d) failed", (ctx)->device)

extern "C" {

int vd_abi_version(void) { return VDMI_ABI_VERSION; }
const char* vd_last_error(void) { return g_err.c_str(); }

int vd_default_cfg(vd_cfg* c) {
    if (!c) return vd_set_error(VD_ERR_ARG, "null cfg");
    memset(c, 0, sizeof *c);
    c->input_h = 640; c->input_w = 640;     // combine_detect.py:860
    c->max_batch = 64;                      // config.ini:35
    c->max_frame_h = 2160; c->max_frame_w = 3840;
    c->precision = VD_PREC_BF16;
    c->max_boxes = 256;
    c->confidence = 0.5f;                   // combine_detect.py:861
    c->nms_iou = 0.4;                       // combine_detect.py:862
    c->mosaic_level = 8;                    // combine_detect.py:249
    c->plate_imgsz = 640;
    c->plate_nc = 1;
    c->plate_conf = 0.5f;                   // combine_detect.py:217
    c->plate_iou = 0.7;                     // ultralytics default [ext]
    c->plate_max_det = 300;                 // ultralytics default [ext]
    return VD_OK;
}

int vd_create(const vd_cfg* cfg, int device, vd_ctx** out) {
    if (!out) return vd_set_error(VD_ERR_ARG, "null out");
    *out = nullptr;
    vd_cfg c;
    if (cfg) c = *cfg; else vd_default_cfg(&c);
    if (c.max_batch <= 0 || c.input_h % 32 || c.input_w % 32 || c.input_h <= 0 || c.input_w <= 0)
        return vd_set_error(VD_ERR_ARG, "cfg: max_batch>0 and input dims multiple of 32 required");
    if (c.precision != VD_PREC_BF16 && c.precision != VD_PREC_FP32 && c.precision != VD_PREC_FP16)
        return vd_set_error(VD_ERR_ARG, "cfg: bad precision");
    if (c.mosaic_level <= 0) c.mosaic_level = 8;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev)
        return vd_set_error(VD_ERR_HIP, "no HIP device %d (count %d)", device, ndev);
    if (hipSetDevice(device) != hipSuccess) return vd_set_error(VD_ERR_HIP, "hipSetDevice(%d)", device);
    Ctx* ctx = new Ctx();
    ctx->cfg = c;
    ctx->device = device;
    ctx->f32 = c.precision == VD_PREC_FP32;
    ctx->f16 = c.precision == VD_PREC_FP16;
    if (hipStreamCreateWithFlags(&ctx->own_stream, hipStreamNonBlocking) != hipSuccess) {
        delete ctx;
        return vd_set_error(VD_ERR_HIP, "hipStreamCreate failed");
    }
    ctx->stream = ctx->own_stream;
    {
        const unsigned hw = std::thread::hardware_concurrency();
        ctx->jpeg_threads = (int)std::max(1u, std::min(16u, hw ? hw : 4u));   // one GPU's host share
    }
    if (hipEventCreateWithFlags(&ctx->jpeg_ev, hipEventDisableTiming) != hipSuccess ||
        hipStreamCreateWithFlags(&ctx->stream2, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&ctx->ev_fork, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&ctx->ev_join, hipEventDisableTiming) != hipSuccess) {
        hipStreamDestroy(ctx->own_stream);
        delete ctx;
        return vd_set_error(VD_ERR_HIP, "stream/event creation failed");
    }
    *out = (vd_ctx*)ctx;
    return VD_OK;
}

int vd_destroy(vd_ctx* h) {
    Ctx* ctx = (Ctx*)h;
    if (!ctx) return VD_OK;
    hipSetDevice(ctx->device);
    hipStreamSynchronize(ctx->stream);
    for (void* p : ctx->allocs) hipFree(p);
    if (ctx->stage_in) hipFree(ctx->stage_in);
    if (ctx->stage_out) hipFree(ctx->stage_out);
    if (ctx->stage_box) hipFree(ctx->stage_box);
    if (ctx->stage_box2) hipFree(ctx->stage_box2);
    if (ctx->mosaic_table) hipFree(ctx->mosaic_table);
    if (ctx->jpeg_dev) hipFree(ctx->jpeg_dev);
    if (ctx->jpeg_planes) hipFree(ctx->jpeg_planes);
    if (ctx->jpeg_host) hipHostFree(ctx->jpeg_host);
    if (ctx->jdec_host) hipHostFree(ctx->jdec_host);
    if (ctx->jdec_dev) hipFree(ctx->jdec_dev);
    if (ctx->jdec_work) hipFree(ctx->jdec_work);
    if (ctx->jenc_dev) hipFree(ctx->jenc_dev);
    if (ctx->jhuf_dev) hipFree(ctx->jhuf_dev);
    if (ctx->jseg_host) hipHostFree(ctx->jseg_host);
    if (ctx->jenc_host) hipHostFree(ctx->jenc_host);
    if (ctx->jpeg_ev) hipEventDestroy(ctx->jpeg_ev);
    for (auto& t : ctx->ev_pool) { hipEventDestroy(t.a); hipEventDestroy(t.b); }
    hipStreamSynchronize(ctx->stream2);
    if (ctx->stream_side) {
        hipStreamSynchronize(ctx->stream_side);
        hipStreamDestroy(ctx->stream_side);
        hipEventDestroy(ctx->ev_side);
    }
    for (hipEvent_t ev : ctx->lane_ev)
        if (ev) hipEventDestroy(ev);
    hipEventDestroy(ctx->ev_fork);
    hipEventDestroy(ctx->ev_join);
    if (ctx->ev_half) hipEventDestroy(ctx->ev_half);
    for (size_t g = 0; g < ctx->group_streams.size(); ++g) {
        hipStreamSynchronize(ctx->group_streams[g]);
        hipStreamDestroy(ctx->group_streams[g]);
        hipEventDestroy(ctx->group_events[g]);
    }
    hipStreamDestroy(ctx->stream2);
    hipStreamDestroy(ctx->own_stream);
    delete ctx;
    return VD_OK;
}

int vd_load_weights(vd_ctx* h, int net, const void* blob, size_t bytes, int fmt) {
    Ctx* ctx = (Ctx*)h;
    VD_ENTRY(ctx);
    if (fmt != VD_WEIGHTS_VDW1) return vd_set_error(VD_ERR_ARG, "unknown weight format %d", fmt);
    if (!blob) return vd_set_error(VD_ERR_ARG, "null weight blob");
    WMap W;
    int rc = vd_parse_vdw1(blob, bytes, W);
    if (rc) return rc;
    if (net == VD_NET_RETINAFACE) {
        if (ctx->face.loaded) return vd_set_error(VD_ERR_STATE, "RetinaFace weights already loaded");
        return vd_build_face(*ctx, W);
    }
    if (net == VD_NET_YOLOV8N) {
        if (ctx->plate.loaded) return vd_set_error(VD_ERR_STATE, "plate weights already loaded");
        return vd_build_plate(*ctx, W);
    }
    return vd_set_error(VD_ERR_ARG, "unknown net %d", net);
}

int vd_set_option(vd_ctx* h, const char* name, int value) {
    Ctx* ctx = (Ctx*)h;
    VD_ENTRY(ctx);
    if (!name) return vd_set_error(VD_ERR_ARG, "null option name");
    struct Opt { const char* n; int VdTune::*f; };
    static const Opt opts[] = {
        {"conv_stream", &VdTune::conv_stream}, {"conv_stream512", &VdTune::conv_stream512},
        {"conv_dual", &VdTune::conv_dual}, {"conv_taps", &VdTune::conv_taps}, {"conv_n192", &VdTune::conv_n192},
        {"conv_small", &VdTune::conv_small}, {"conv_big", &VdTune::conv_big},
        {"conv_big_kmin", &VdTune::conv_big_kmin}, {"stream_ntt", &VdTune::stream_ntt},
        {"lb_pair", &VdTune::lb_pair}, {"mosaic_map", &VdTune::mosaic_map}, {"mosaic_nt", &VdTune::mosaic_nt}, {"mosaic_cells", &VdTune::mosaic_cells}, {"mosaic_fused", &VdTune::mosaic_fused}, {"mosaic_rows", &VdTune::mosaic_rows}, {"mosaic_gather", &VdTune::mosaic_gather}, {"block_fuse", &VdTune::block_fuse},
        {"chain", &VdTune::chain}, {"stem_pool", &VdTune::stem_pool}, {"ssh_fuse", &VdTune::ssh_fuse},
        {"plate_s2d", &VdTune::plate_s2d}, {"f32_split", &VdTune::f32_split},
        {"x6_small_k", &VdTune::x6_small_k}, {"x6_small_tiles", &VdTune::x6_small_tiles},
        {"x6_stream", &VdTune::x6_stream}, {"x6_small_k2", &VdTune::x6_small_k2}, {"x6_bn256", &VdTune::x6_bn256},
        {"x6_exact", &VdTune::x6_exact}, {"x6_mid", &VdTune::x6_mid}, {"block_fuse32", &VdTune::block_fuse32}, {"x6_mf32", &VdTune::x6_mf32}, {"x6_tail", &VdTune::x6_tail}, {"x6_stream_silu", &VdTune::x6_stream_silu}, {"x6_stream_rl", &VdTune::x6_stream_rl}, {"x6_gemm_uni", &VdTune::x6_gemm_uni}, {"x6_halo_1b", &VdTune::x6_halo_1b}, {"x6_slots", &VdTune::x6_slots}, {"x6_halo", &VdTune::x6_halo}, {"x6_halo_narrow", &VdTune::x6_halo_narrow}, {"x6_halo_s2", &VdTune::x6_halo_s2}, {"x6_adepth", &VdTune::x6_adepth}, {"x6_gemm1x1", &VdTune::x6_gemm1x1}, {"x6_taps", &VdTune::x6_taps}, {"x6_halo_tr", &VdTune::x6_halo_tr}, {"x6_tr_epi", &VdTune::x6_tr_epi}, {"x6_halo_dma", &VdTune::x6_halo_dma}, {"x6_halo_pf", &VdTune::x6_halo_pf}, {"x6_halo_n64", &VdTune::x6_halo_n64}, {"x6_gemm_pf", &VdTune::x6_gemm_pf}, {"x6_stream256", &VdTune::x6_stream256}, {"plate_stage", &VdTune::plate_stage}, {"plate_detect_early", &VdTune::plate_detect_early}, {"mosaic_early", &VdTune::mosaic_early}, {"ssh_side", &VdTune::ssh_side}, {"face_groups", &VdTune::face_groups}, {"plate_s2d32", &VdTune::plate_s2d32}, {"det_group", &VdTune::det_group}, {"chain_gpw", &VdTune::chain_gpw}, {"block32_xd", &VdTune::block32_xd}, {"block32_pipe", &VdTune::block32_pipe}, {"x6_one", &VdTune::x6_one},
        {"jenc_gpu", &VdTune::jenc_gpu}, {"jdec_gpu", &VdTune::jdec_gpu}, {"jdec_chunk", &VdTune::jdec_chunk}, {"jdec_sync", &VdTune::jdec_sync}, {"jdec_group", &VdTune::jdec_group},
    };
    for (const Opt& o : opts)
        if (strcmp(o.n, name) == 0) {
            if (!strcmp(name, "stream_ntt") && value != 8 && value != 16)
                return vd_set_error(VD_ERR_ARG, "stream_ntt must be 8 or 16");
            ctx->tune.*(o.f) = value;
            return VD_OK;
        }
    return vd_set_error(VD_ERR_ARG, "unknown option '%s'", name);
}

int vdt_set_debug(vd_ctx* h, const char* name, int value) {
    Ctx* ctx = (Ctx*)h;
    VD_ENTRY(ctx);
    if (!name) return vd_set_error(VD_ERR_ARG, "null debug switch name");
    // timing-only stage skips: results are WRONG while set (tools/x6bench, tools/runs)
    if (!strcmp(name, "x6_dbg")) { ctx->tune.x6_dbg = value; return VD_OK; }
    if (!strcmp(name, "block32_dbg")) { ctx->tune.block32_dbg = value; return VD_OK; }
    return vd_set_error(VD_ERR_ARG, "unknown debug switch '%s'", name);
}

int vd_set_stream(vd_ctx* h, void* s) {
    Ctx* ctx = (Ctx*)h;
    VD_ENTRY(ctx);
    ctx->stream = s ? (hipStream_t)s : ctx->own_stream;
    return VD_OK;
}

void* vd_get_stream(vd_ctx* h) { return h ? (void*)((Ctx*)h)->stream : nullptr; }

int vd_sync(vd_ctx* h) {
    Ctx* ctx = (Ctx*)h;
    VD_ENTRY(ctx);
    VD_CHECK_HIP(hipStreamSynchronize(ctx->stream));
    return VD_OK;
}

int vd_detect(vd_ctx* h, const uint8_t* frames, int n, int fh, int fw, size_t pitch, int where, vd_boxes* faces) {
    Ctx* ctx = (Ctx*)h;
    VD_ENTRY(ctx);
    if (!ctx->face.loaded) return vd_set_error(VD_ERR_STATE, "RetinaFace weights not loaded");
    int rc = ctx->check_frames(n, fh, fw, pitch);
    if (rc) return rc;
    BoxTargets t;
    rc = ctx->box_targets(faces, n, t);
    if (rc) return rc;
    const uint8_t* d = ctx->frames_to_device(frames, n, fh, pitch, where, &rc);
    if (rc) return rc;
    if ((rc = ctx->face_letterbox(d, n, fh, fw, pitch))) return rc;
    if ((rc = ctx->face_forward(n))) return rc;
    if ((rc = ctx->face_post(n, fh, fw, t))) return rc;
    return ctx->box_finish(faces, n, t);
}

int vd_detect_plates(vd_ctx* h, const uint8_t* frames, int n, int fh, int fw, size_t pitch, int where,
                     vd_boxes* plates) {
    Ctx* ctx = (Ctx*)h;
    VD_ENTRY(ctx);
    if (!ctx->plate.loaded) return vd_set_error(VD_ERR_STATE, "plate weights not loaded");
    int rc = ctx->check_frames(n, fh, fw, pitch);
    if (rc) return rc;
    BoxTargets t;
    rc = ctx->box_targets(plates, n, t);
    if (rc) return rc;
    const uint8_t* d = ctx->frames_to_device(frames, n, fh, pitch, where, &rc);
    if (rc) return rc;
    if ((rc = vd_plate_forward(*ctx, d, n, fh, fw, pitch))) return rc;
    if ((rc = vd_plate_post(*ctx, n, fh, fw, t))) return rc;
    return ctx->box_finish(plates, n, t);
}

int vd_mosaic(vd_ctx* h, const uint8_t* in, uint8_t* out, int n, int fh, int fw, size_t pitch, int where,
              const vd_boxes* boxes, int level, int mode) {
    Ctx* ctx = (Ctx*)h;
    VD_ENTRY(ctx);
    if (mode != VD_MOSAIC_OUT_OF_PLACE) return vd_set_error(VD_ERR_ARG, "unsupported mosaic mode %d", mode);
    if (!in || !out || !boxes || !boxes->count || !boxes->xyxy || boxes->cap <= 0)
        return vd_set_error(VD_ERR_ARG, "vd_mosaic: null argument");
    if (n <= 0 || fh <= 0 || fw <= 0 || pitch < (size_t)fw * 3 || level <= 0)
        return vd_set_error(VD_ERR_ARG, "vd_mosaic: bad geometry");
    if ((const void*)in == (const void*)out ||
        (where == VD_DEVICE && vd_ranges_overlap(in, out, (size_t)n * fh * pitch)))
        return vd_set_error(VD_ERR_ARG, "vd_mosaic: out-of-place only (out must not overlap in)");
    int rc = VD_OK;
    const uint8_t* din = in;
    uint8_t* dout = out;
    size_t bytes = (size_t)n * fh * pitch;
    if (where == VD_HOST) {
        if ((rc = ctx->ensure_staging(&ctx->stage_in, &ctx->stage_in_bytes, bytes))) return rc;
        if ((rc = ctx->ensure_staging(&ctx->stage_out, &ctx->stage_out_bytes, bytes))) return rc;
        VD_CHECK_HIP(hipMemcpyAsync(ctx->stage_in, in, bytes, hipMemcpyHostToDevice, ctx->stream));
        din = (const uint8_t*)ctx->stage_in;
        dout = (uint8_t*)ctx->stage_out;
    }
    const int* cnt = boxes->count;
    const int* xy = boxes->xyxy;
    if (boxes->where == VD_HOST)   // a count past cap means boxes the caller does not hold: never skip them silently
        for (int i = 0; i < n; ++i)
            if (boxes->count[i] > boxes->cap)
                return vd_set_error(VD_ERR_CAPACITY, "vd_mosaic: frame %d has count %d > cap %d (read the complete "
                                    "list with vd_read_boxes)", i, boxes->count[i], boxes->cap);
    if (boxes->where == VD_HOST) {
        size_t nb = (size_t)n * boxes->cap;
        if ((rc = ctx->ensure_staging(&ctx->stage_box2, &ctx->stage_box2_bytes, n * 4 + nb * 16 + 16))) return rc;
        int* dc = (int*)ctx->stage_box2;
        int* dx = dc + ((n + 3) / 4) * 4;
        VD_CHECK_HIP(hipMemcpyAsync(dc, boxes->count, n * 4, hipMemcpyHostToDevice, ctx->stream));
        VD_CHECK_HIP(hipMemcpyAsync(dx, boxes->xyxy, nb * 16, hipMemcpyHostToDevice, ctx->stream));
        cnt = dc;
        xy = dx;
    }
    if ((rc = ctx->launch_mosaic(din, dout, n, fh, fw, pitch, cnt, xy, boxes->cap, nullptr, nullptr, 0, level)))
        return rc;
    if (where == VD_HOST) {
        VD_CHECK_HIP(hipMemcpyAsync(out, dout, bytes, hipMemcpyDeviceToHost, ctx->stream));
        VD_CHECK_HIP(hipStreamSynchronize(ctx->stream));
    } else if (boxes->where == VD_HOST) {
        VD_CHECK_HIP(hipStreamSynchronize(ctx->stream));   // staging reused by the next call
    }
    return VD_OK;
}

int vd_process(vd_ctx* h, const uint8_t* in, uint8_t* out, int n, int fh, int fw, size_t pitch, int where,
               int flags, vd_boxes* faces, vd_boxes* plates) {
    Ctx* ctx = (Ctx*)h;
    VD_ENTRY(ctx);
    const bool do_faces = flags & VD_PROC_FACES, do_plates = flags & VD_PROC_PLATES;
    const bool do_mosaic = flags & VD_PROC_MOSAIC, mosaic_plates = flags & VD_PROC_MOSAIC_PLATES;
    if (do_faces && !ctx->face.loaded) return vd_set_error(VD_ERR_STATE, "RetinaFace weights not loaded");
    if (do_plates && !ctx->plate.loaded) return vd_set_error(VD_ERR_STATE, "plate weights not loaded");
    if (mosaic_plates && !do_plates) return vd_set_error(VD_ERR_ARG, "MOSAIC_PLATES needs PLATES");
    if (do_mosaic && !out) return vd_set_error(VD_ERR_ARG, "MOSAIC needs an output buffer");
    int rc = ctx->check_frames(n, fh, fw, pitch);
    if (rc) return rc;
    // the mosaic is out of place (combine_detect.py:142 blurs a copy; each box reads the
    // previous box's output, :247-249): its one-launch output pass gathers cell colours
    // from `in` anywhere in the frame while other workgroups write `out`, so device
    // frames that overlap would race (host frames are staged in separate buffers)
    if (do_mosaic && where == VD_DEVICE && vd_ranges_overlap(in, out, (size_t)n * fh * pitch))
        return vd_set_error(VD_ERR_ARG, "vd_process: MOSAIC is out-of-place (out must not overlap in)");
    BoxTargets tf{}, tp{};
    if (do_faces && (rc = ctx->box_targets(faces, n, tf))) return rc;
    if (do_plates && plates) {   // plate box staging must not alias the face staging
        if (!plates->count || !plates->xyxy || plates->cap <= 0)
            return vd_set_error(VD_ERR_ARG, "vd_boxes needs count, xyxy, cap>0");
        if (plates->where == VD_DEVICE) {
            tp.cap = plates->cap; tp.count = plates->count; tp.xyxy = plates->xyxy; tp.xyxy_f = plates->xyxy_f;
            tp.score = plates->score; tp.label = plates->label;
        } else if ((rc = ctx->host_box_staging(&ctx->stage_box2, &ctx->stage_box2_bytes, plates->cap, n, tp))) {
            return rc;
        }
    }
    const uint8_t* d = ctx->frames_to_device(in, n, fh, pitch, where, &rc);
    if (rc) return rc;
    // Face and plate branches run concurrently (the reference submits them to two
    // threads, combine_detect.py:214-217): plates on stream2, forked/joined by events.
    const bool fork = do_faces && do_plates;
    hipStream_t plate_stream = ctx->stream2;
    // Both canvases from one read of the frames where the geometry allows (pre.hip
    // letterbox_s2d_pair_kernel); the plate branch then forks after it.
    bool paired = false;
    if (fork) {
        LetterboxArgs fa, pa;
        ctx->face_letterbox_args(d, n, fh, fw, pitch, &fa);
        if (ctx->tune.lb_pair && vd_plate_letterbox_args(*ctx, d, n, fh, fw, pitch, &pa) == VD_OK &&
            vd_letterbox_pair_ok(fa, pa)) {
            ctx->t_begin(2, (double)n * (fa.nh * (double)fw * 3 + (double)(fa.oh / 2 + 1) * (fa.ow / 2 + 1) * (fa.out_f32 ? 64 : 32) +
                                         (double)(pa.oh / 2 + 1) * (pa.ow / 2 + 1) * (pa.out_f32 ? 64 : 32)));
            hipError_t e = vd_launch_letterbox_pair(fa, pa, ctx->stream);
            ctx->t_end();
            if (e != hipSuccess) return vd_set_error(VD_ERR_HIP, "letterbox pair: %s", hipGetErrorString(e));
            paired = true;
        }
    }
    // The plate branch may be held back until face stage `plate_stage` has been issued
    // (its HBM-bound convs then overlap the MFMA-bound late face layers).
    const int ps = ctx->tune.plate_stage;
    ctx->fork_at = -1;
    if (fork && ps > 0) {
        ctx->fork_at = ps >= 5 ? (int)ctx->face.net.ops.size() : ctx->face.net.stage_end[std::min(ps, 4)];
        if (ctx->fork_at <= 0) ctx->fork_at = -1;
    }
    if (fork && ctx->fork_at < 0) {
        VD_CHECK_HIP(hipEventRecord(ctx->ev_fork, ctx->stream));
        VD_CHECK_HIP(hipStreamWaitEvent(plate_stream, ctx->ev_fork, 0));
    }
    if (do_faces) {
        if (!paired && (rc = ctx->face_letterbox(d, n, fh, fw, pitch))) return rc;
        if ((rc = ctx->face_forward(n))) return rc;
        if (ctx->fork_at > 0) {
            ctx->fork_at = -1;
            VD_CHECK_HIP(hipStreamWaitEvent(plate_stream, ctx->ev_fork, 0));
        }
        if ((rc = ctx->face_post(n, fh, fw, tf))) return rc;
    }
    if (do_plates) {
        hipStream_t main = ctx->stream;
        if (fork) ctx->stream = plate_stream;
        rc = vd_plate_forward(*ctx, d, n, fh, fw, pitch, paired);
        if (!rc) rc = vd_plate_post(*ctx, n, fh, fw, tp);
        ctx->stream = main;
        if (rc) return rc;
    }
    // the mosaic reads plate boxes only with MOSAIC_PLATES (the reference discards them,
    // combine_detect.py:239): otherwise it runs on the face stream before the plate branch
    // joins, beside the branch's last launches (option mosaic_early)
    const bool mosaic_first = do_mosaic && fork && !mosaic_plates && ctx->tune.mosaic_early;
    auto mosaic = [&]() -> int {
        uint8_t* dout = out;
        size_t bytes = (size_t)n * fh * pitch;
        if (where == VD_HOST) {
            int r = ctx->ensure_staging(&ctx->stage_out, &ctx->stage_out_bytes, bytes);
            if (r) return r;
            dout = (uint8_t*)ctx->stage_out;
        }
        // every kept box, from the library's complete keep lists (the caller's arrays
        // may hold fewer: cap), faces in NMS order then plates (combine_detect.py:241-249)
        const PostScratch& fp = ctx->face.post;
        const PostScratch& pp = ctx->plate.post;
        int r = ctx->launch_mosaic(d, dout, n, fh, fw, pitch, do_faces ? fp.kcount : nullptr,
                                   do_faces ? fp.kxyxy : nullptr, do_faces ? fp.kcap : 0,
                                   mosaic_plates ? pp.kcount : nullptr, mosaic_plates ? pp.kxyxy : nullptr,
                                   mosaic_plates ? pp.kcap : 0, ctx->cfg.mosaic_level);
        if (r) return r;
        if (where == VD_HOST) VD_CHECK_HIP(hipMemcpyAsync(out, dout, bytes, hipMemcpyDeviceToHost, ctx->stream));
        return VD_OK;
    };
    if (mosaic_first && (rc = mosaic())) return rc;
    if (fork) {
        VD_CHECK_HIP(hipEventRecord(ctx->ev_join, plate_stream));
        VD_CHECK_HIP(hipStreamWaitEvent(ctx->stream, ctx->ev_join, 0));
    }
    if (do_mosaic && !mosaic_first && (rc = mosaic())) return rc;
    int rc2 = VD_OK;
    if (do_faces) rc2 = ctx->box_finish(faces, n, tf);
    if (do_plates) {
        int rc3 = ctx->box_finish(plates, n, tp);
        if (!rc2) rc2 = rc3;
    }
    if (where == VD_HOST) VD_CHECK_HIP(hipStreamSynchronize(ctx->stream));
    return rc2;
}

int vd_read_boxes(vd_ctx* h, int net, int n, vd_boxes* out) {
    Ctx* ctx = (Ctx*)h;
    VD_ENTRY(ctx);
    const PostScratch* ps = net == VD_NET_RETINAFACE ? &ctx->face.post : (net == VD_NET_YOLOV8N ? &ctx->plate.post : nullptr);
    if (!ps) return vd_set_error(VD_ERR_ARG, "unknown net %d", net);
    if (!ps->kcount) return vd_set_error(VD_ERR_STATE, "net %d not loaded", net);
    if (!out || !out->count || !out->xyxy || out->cap <= 0) return vd_set_error(VD_ERR_ARG, "vd_boxes needs count, xyxy, cap>0");
    if (n <= 0 || n > ps->kn) return vd_set_error(VD_ERR_ARG, "n=%d outside [1, %d frames of the last call]", n, ps->kn);
    const hipMemcpyKind kind = out->where == VD_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
    const int w = std::min(out->cap, ps->kcap);   // boxes per frame copied (beyond kcap nothing is ever kept)
    const size_t dp = (size_t)out->cap, sp = (size_t)ps->kcap;
    VD_CHECK_HIP(hipMemcpyAsync(out->count, ps->kcount, (size_t)n * 4, kind, ctx->stream));
    VD_CHECK_HIP(hipMemcpy2DAsync(out->xyxy, dp * 16, ps->kxyxy, sp * 16, (size_t)w * 16, n, kind, ctx->stream));
    if (out->xyxy_f)
        VD_CHECK_HIP(hipMemcpy2DAsync(out->xyxy_f, dp * 16, ps->kxyxy_f, sp * 16, (size_t)w * 16, n, kind, ctx->stream));
    if (out->score)
        VD_CHECK_HIP(hipMemcpy2DAsync(out->score, dp * 4, ps->kscore, sp * 4, (size_t)w * 4, n, kind, ctx->stream));
    if (out->label)
        VD_CHECK_HIP(hipMemcpy2DAsync(out->label, dp * 4, ps->klabel, sp * 4, (size_t)w * 4, n, kind, ctx->stream));
    if (out->where == VD_HOST) VD_CHECK_HIP(hipStreamSynchronize(ctx->stream));
    return VD_OK;
}

int vd_timing_enable(vd_ctx* h, int on) {
    Ctx* ctx = (Ctx*)h;
    VD_ENTRY(ctx);
    ctx->timing = on != 0;
    return VD_OK;
}

int vd_timing_reset(vd_ctx* h) {
    Ctx* ctx = (Ctx*)h;
    VD_ENTRY(ctx);
    VD_CHECK_HIP(hipStreamSynchronize(ctx->stream));
    ctx->ev_used = 0;
    return VD_OK;
}

int vd_timing_read(vd_ctx* h, int fam, double* ms, int64_t* launches, double* work) {
    Ctx* ctx = (Ctx*)h;
    VD_ENTRY(ctx);
    VD_CHECK_HIP(hipStreamSynchronize(ctx->stream));
    double tot = 0, wk = 0;
    int64_t cnt = 0;
    for (size_t i = 0; i < ctx->ev_used; ++i) {
        const TimedEv& t = ctx->ev_pool[i];
        if (t.fam != fam) continue;
        float e = 0.f;
        VD_CHECK_HIP(hipEventElapsedTime(&e, t.a, t.b));
        tot += e;
        wk += t.work;
        ++cnt;
    }
    if (ms) *ms = tot;
    if (launches) *launches = cnt;
    if (work) *work = wk;
    return VD_OK;
}

// ---- test hooks ----
int vdt_letterbox(vd_ctx* h, const uint8_t* frames, int n, int fh, int fw, size_t pitch, int where, float* out,
                  int cpad) {
    Ctx* ctx = (Ctx*)h;
    VD_ENTRY(ctx);
    if (!ctx->face.loaded) return vd_set_error(VD_ERR_STATE, "RetinaFace weights not loaded");
    int rc = ctx->check_frames(n, fh, fw, pitch);
    if (rc) return rc;
    const uint8_t* d = ctx->frames_to_device(frames, n, fh, pitch, where, &rc);
    if (rc) return rc;
    if ((rc = ctx->face_letterbox(d, n, fh, fw, pitch))) return rc;
    const Act& in = ctx->face.input;
    size_t px = (size_t)n * in.h * in.w;
    std::vector<uint16_t> hb;
    std::vector<float> hf;
    VD_CHECK_HIP(hipStreamSynchronize(ctx->stream));
    if (in.f32) {
        hf.resize(px * in.c);
        VD_CHECK_HIP(hipMemcpy(hf.data(), in.p, hf.size() * 4, hipMemcpyDeviceToHost));
    } else {
        hb.resize(px * in.c);
        VD_CHECK_HIP(hipMemcpy(hb.data(), in.p, hb.size() * 2, hipMemcpyDeviceToHost));
    }
    if (ctx->face.s2d) {   // unpack the space-to-depth canvas back to [n][H][W][cpad]
        const int H = ctx->face.in_h, W = ctx->face.in_w;
        for (int f = 0; f < n; ++f)
            for (int y = 0; y < H; ++y)
                for (int x = 0; x < W; ++x)
                    for (int c = 0; c < cpad; ++c) {
                        float v = 0.f;
                        if (c < 3) {
                            const int Y = (y + 1) >> 1, X = (x + 1) >> 1, s = ((y + 1) & 1) * 2 + ((x + 1) & 1);
                            const size_t i = (((size_t)f * in.h + Y) * in.w + X) * in.c + s * 4 + c;
                            if (ctx->f32) {                 // fused fp32 stem: fp16 canvas
                                v = from_half(true, hb[i]);
                            } else {
                                uint32_t u = (uint32_t)hb[i] << 16;
                                memcpy(&v, &u, 4);
                            }
                        }
                        out[(((size_t)f * H + y) * W + x) * cpad + c] = v;
                    }
        return VD_OK;
    }
    for (size_t i = 0; i < px; ++i)
        for (int c = 0; c < cpad; ++c) {
            float v = 0.f;
            if (c < in.c) {
                if (in.f32) v = hf[i * in.c + c];
                else v = from_half(ctx->f16, hb[i * in.c + c]);
            }
            out[i * cpad + c] = v;
        }
    return VD_OK;
}

int vdt_forward_heads(vd_ctx* h, const uint8_t* frames, int n, int fh, int fw, size_t pitch, int where, float* loc,
                      float* conf, float* landm) {
    Ctx* ctx = (Ctx*)h;
    VD_ENTRY(ctx);
    if (!ctx->face.loaded) return vd_set_error(VD_ERR_STATE, "RetinaFace weights not loaded");
    int rc = ctx->check_frames(n, fh, fw, pitch);
    if (rc) return rc;
    const uint8_t* d = ctx->frames_to_device(frames, n, fh, pitch, where, &rc);
    if (rc) return rc;
    if ((rc = ctx->face_letterbox(d, n, fh, fw, pitch))) return rc;
    if ((rc = ctx->face_forward(n))) return rc;
    VD_CHECK_HIP(hipStreamSynchronize(ctx->stream));
    const int A = ctx->face.A;
    for (int l = 0; l < 3; ++l) {
        const Act& hd = ctx->face.heads[l];
        std::vector<float> buf((size_t)n * hd.h * hd.w * 32);
        VD_CHECK_HIP(hipMemcpy(buf.data(), hd.p, buf.size() * 4, hipMemcpyDeviceToHost));
        for (int b = 0; b < n; ++b)
            for (int px = 0; px < hd.h * hd.w; ++px)
                for (int k = 0; k < 2; ++k) {
                    const float* src = &buf[((size_t)b * hd.h * hd.w + px) * 32];
                    size_t a = (size_t)b * A + ctx->face.loff[l] + px * 2 + k;
                    if (loc) for (int j = 0; j < 4; ++j) loc[a * 4 + j] = src[4 * k + j];
                    if (conf) for (int j = 0; j < 2; ++j) conf[a * 2 + j] = src[8 + 2 * k + j];
                    if (landm) for (int j = 0; j < 10; ++j) landm[a * 10 + j] = src[12 + 10 * k + j];
                }
    }
    return VD_OK;
}

int vdt_postprocess(vd_ctx* h, const float* loc, const float* conf, int n, const int32_t* img_hw, vd_boxes* faces) {
    Ctx* ctx = (Ctx*)h;
    VD_ENTRY(ctx);
    if (!ctx->face.loaded) return vd_set_error(VD_ERR_STATE, "RetinaFace weights not loaded");
    if (n <= 0 || n > ctx->cfg.max_batch || !loc || !conf || !img_hw) return vd_set_error(VD_ERR_ARG, "vdt_postprocess args");
    for (int i = 1; i < n; ++i)
        if (img_hw[2 * i] != img_hw[0] || img_hw[2 * i + 1] != img_hw[1])
            return vd_set_error(VD_ERR_ARG, "vdt_postprocess: frames of one call share a size");
    const int A = ctx->face.A;
    for (int l = 0; l < 3; ++l) {
        const Act& hd = ctx->face.heads[l];
        std::vector<float> buf((size_t)n * hd.h * hd.w * 32, 0.f);
        for (int b = 0; b < n; ++b)
            for (int px = 0; px < hd.h * hd.w; ++px)
                for (int k = 0; k < 2; ++k) {
                    float* dst = &buf[((size_t)b * hd.h * hd.w + px) * 32];
                    size_t a = (size_t)b * A + ctx->face.loff[l] + px * 2 + k;
                    for (int j = 0; j < 4; ++j) dst[4 * k + j] = loc[a * 4 + j];
                    for (int j = 0; j < 2; ++j) dst[8 + 2 * k + j] = conf[a * 2 + j];
                }
        VD_CHECK_HIP(hipMemcpy(hd.p, buf.data(), buf.size() * 4, hipMemcpyHostToDevice));
    }
    BoxTargets t;
    int rc = ctx->box_targets(faces, n, t);
    if (rc) return rc;
    if ((rc = ctx->face_post(n, img_hw[0], img_hw[1], t))) return rc;
    rc = ctx->box_finish(faces, n, t);
    VD_CHECK_HIP(hipStreamSynchronize(ctx->stream));
    return rc;
}

int vdt_conv2d(vd_ctx* h, const float* x, int n, int xh, int xw, int cin, const float* wgt, int cout, int kh, int kw,
               int stride, int pad, const float* scale, const float* shift, int act, float slope, const float* res,
               int res_mode, float* y, int* oh_out, int* ow_out) {
    Ctx* ctx = (Ctx*)h;
    VD_ENTRY(ctx);
    if (n <= 0 || xh <= 0 || xw <= 0 || cin <= 0 || cout <= 0 || kh <= 0 || kw <= 0 || stride <= 0 || pad < 0)
        return vd_set_error(VD_ERR_ARG, "vdt_conv2d: bad shape");
    Conv cv{};
    cv.cin = cin; cv.cout = cout; cv.kh = kh; cv.kw = kw; cv.stride = stride; cv.pad = pad; cv.act = act;
    cv.slope = slope;
    std::vector<float> w(wgt, wgt + (size_t)cout * cin * kh * kw);
    std::vector<float> sc(scale, scale + cout), sh(shift, shift + cout);
    const size_t nalloc = ctx->allocs.size();
    int rc = ctx->upload_conv(cv, w, sc, sh);
    if (rc) return rc;
    const int oh = (xh + 2 * pad - kh) / stride + 1, ow = (xw + 2 * pad - kw) / stride + 1;
    const int es = ctx->f32 ? 4 : 2;
    const int ldx = cv.cin_pad;
    const int ldy = (cout + 7) / 8 * 8;
    std::vector<char> xb((size_t)n * xh * xw * ldx * es, 0), rb;
    for (size_t p = 0; p < (size_t)n * xh * xw; ++p)
        for (int c = 0; c < cin; ++c) {
            float v = x[p * cin + c];
            if (ctx->f32) memcpy(&xb[(p * ldx + c) * 4], &v, 4);
            else { uint16_t b = to_half(ctx->f16, v); memcpy(&xb[(p * ldx + c) * 2], &b, 2); }
        }
    void *dx = nullptr, *dy = nullptr, *dr = nullptr;
    if ((rc = ctx->dalloc(&dx, xb.size()))) return rc;
    if ((rc = ctx->dalloc(&dy, (size_t)n * oh * ow * ldy * 4))) return rc;   // f32 output
    VD_CHECK_HIP(hipMemcpy(dx, xb.data(), xb.size(), hipMemcpyHostToDevice));
    if (res && res_mode) {
        rb.assign((size_t)n * oh * ow * ldy * es, 0);
        for (size_t p = 0; p < (size_t)n * oh * ow; ++p)
            for (int c = 0; c < cout; ++c) {
                float v = res[p * cout + c];
                if (ctx->f32) memcpy(&rb[(p * ldy + c) * 4], &v, 4);
                else { uint16_t b = to_half(ctx->f16, v); memcpy(&rb[(p * ldy + c) * 2], &b, 2); }
            }
        if ((rc = ctx->dalloc(&dr, rb.size()))) return rc;
        VD_CHECK_HIP(hipMemcpy(dr, rb.data(), rb.size(), hipMemcpyHostToDevice));
    }
    ConvArgs a{};
    a.x = dx; a.xh = xh; a.xw = xw; a.ldx = ldx; a.xcoff = 0;
    a.w = cv.w; a.scale = cv.scale; a.shift = cv.shift;
    a.res = dr; a.res_ld = ldy; a.res_coff = 0; a.res_up = 0; a.rh = oh; a.rw = ow;
    a.res_mode = dr ? res_mode : VD_RES_NONE;
    a.y = dy; a.yh = oh; a.yw = ow; a.ldy = ldy; a.ycoff = 0;
    a.B = n; a.cin_pad = cv.cin_pad; a.cout = cout; a.kpad = cv.kpad;
    a.kh = kh; a.kw = kw; a.stride = stride; a.pad = pad; a.M = n * oh * ow;
    a.act = act; a.slope = slope; a.out_f32 = 1; a.f16 = ctx->f16 ? 1 : 0;
    a.tune = &ctx->tune;
    a.wx3 = cv.wx3;
    a.scale_x = cv.scale_x;
    a.f32_split = cv.split;
    // fp16-pair plan: the input's per-frame max |x| as a producer would have left it,
    // and the output's slots, checked below against the host max of the result
    unsigned* dm = nullptr;
    const bool ranged = cv.split == 2;
    if (ranged) {
        std::vector<unsigned> xm(2 * n, 0u);
        for (int b = 0; b < n; ++b) {
            float m = 0.f;
            for (size_t i = (size_t)b * xh * xw * cin; i < (size_t)(b + 1) * xh * xw * cin; ++i) m = std::max(m, std::fabs(x[i]));
            memcpy(&xm[b], &m, 4);
        }
        if ((rc = ctx->dalloc((void**)&dm, xm.size() * 4))) return rc;
        VD_CHECK_HIP(hipMemcpy(dm, xm.data(), xm.size() * 4, hipMemcpyHostToDevice));
        a.xmax = dm;
        a.ymax = dm + n;
    }
    hipError_t e = vd_launch_conv(a, ctx->f32, ctx->stream);
    if (e != hipSuccess) return vd_set_error(VD_ERR_HIP, "conv launch: %s", hipGetErrorString(e));
    VD_CHECK_HIP(hipStreamSynchronize(ctx->stream));
    std::vector<float> yb((size_t)n * oh * ow * ldy);
    VD_CHECK_HIP(hipMemcpy(yb.data(), dy, yb.size() * 4, hipMemcpyDeviceToHost));
    for (size_t p = 0; p < (size_t)n * oh * ow; ++p)
        for (int c = 0; c < cout; ++c) y[p * cout + c] = yb[p * ldy + c];
    if (ranged && cv.wx3) {
        std::vector<float> ym(n);
        VD_CHECK_HIP(hipMemcpy(ym.data(), dm + n, n * 4, hipMemcpyDeviceToHost));
        for (int b = 0; b < n; ++b) {
            float m = 0.f;
            for (size_t i = (size_t)b * oh * ow * cout; i < (size_t)(b + 1) * oh * ow * cout; ++i) m = std::max(m, std::fabs(y[i]));
            if (m != ym[b]) {
                for (size_t i = nalloc; i < ctx->allocs.size(); ++i) hipFree(ctx->allocs[i]);
                ctx->allocs.resize(nalloc);
                return vd_set_error(VD_ERR_HIP, "frame %d: output max slot %g, host max %g", b, ym[b], m);
            }
        }
    }
    if (oh_out) *oh_out = oh;
    if (ow_out) *ow_out = ow;
    // release this call's temporaries
    for (size_t i = nalloc; i < ctx->allocs.size(); ++i) hipFree(ctx->allocs[i]);
    ctx->allocs.resize(nalloc);
    return VD_OK;
}

}  // extern "C"
