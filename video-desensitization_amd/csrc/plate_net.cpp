// plate_net.cpp — YOLOv8n plate detector (ultralytics [ext], combine_detect.py:9,217,872).
//
// The reference calls `plate_detector(batch, verbose=False, conf=0.5)` on an
// ultralytics YOLO model (best.pt, architecture YOLOv8n by SURVEY.md §8a row 11).
// Rebuilt on the same conv/pool/upsample kernels as RetinaFace, NHWC, with the
// ultralytics module tree as state_dict keys (model.<i>.conv/bn, C2f cv1/cv2/m.<j>,
// SPPF, Detect cv2/cv3/dfl). Concats are free: producers write channel slices of
// one buffer (C2f chunk/concat, SPPF concat, the four neck Concats), the
// Bottleneck shortcut is a post-activation residual, Upsample writes straight
// into its Concat slice, and Detect's first box/cls convs (same input) are one
// conv with Cout = 64 + 64. Letterbox geometry depends on the frame aspect
// (auto stride-32 padding), so plans are built lazily per canvas size over
// buffers allocated once for the imgsz x imgsz canvas.
#include "nets.h"
#include "vd_math.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <string>
#include <vector>

namespace {
constexpr float YOLO_BN_EPS = 1e-3f;   // ultralytics initialize_weights sets BatchNorm eps = 1e-3 [ext]
constexpr float MAX_WH = 7680.f;       // ultralytics non_max_suppression max_wh [ext]

struct Buf { const char* name; int div; int c; };
// activation buffers: spatial size = canvas / div
const Buf kBufs[] = {
    {"A0", 2, 16},   {"A1", 4, 32},   {"C2", 4, 48},   {"T2", 4, 16},   {"A2", 4, 32},
    {"A3", 8, 64},   {"C4", 8, 128},  {"T4", 8, 32},   {"cat14", 8, 192},
    {"A5", 16, 128}, {"C6", 16, 256}, {"T6", 16, 64},  {"cat11", 16, 384},
    {"A7", 32, 256}, {"C8", 32, 384}, {"T8", 32, 128}, {"A8", 32, 256}, {"S9", 32, 512}, {"cat20", 32, 384},
    {"C12", 16, 192}, {"T12", 16, 64}, {"cat17", 16, 192},
    {"C15", 8, 96},  {"T15", 8, 32},  {"P3", 8, 64},
    {"C18", 16, 192}, {"T18", 16, 64}, {"P4", 16, 128},
    {"C21", 32, 384}, {"T21", 32, 128}, {"P5", 32, 256},
    {"D0_0", 8, 128}, {"D1_0", 8, 128}, {"D0_1", 16, 128}, {"D1_1", 16, 128}, {"D0_2", 32, 128}, {"D1_2", 32, 128},
};

const Act* find_buf(const PlateNet& P, const std::string& n) {
    for (auto& b : P.bufs)
        if (b.first == n) return &b.second;
    return nullptr;
}

int conv_of(const PlateNet& P, const std::string& n) {
    for (auto& c : P.conv_idx)
        if (c.first == n) return c.second;
    return -1;
}

// ultralytics Conv: Conv2d(k, s, autopad k//2, bias=False) + BN + SiLU
int yconv(Ctx& c, const WMap& W, const std::string& pre, int stride) {
    const HT* w = find_t(W, pre + ".conv.weight");
    if (!w) return vd_set_error(VD_ERR_WEIGHTS, "missing %s.conv.weight", pre.c_str());
    int idx;
    int rc = c.make_conv_bn(W, pre + ".conv.weight", pre + ".bn", YOLO_BN_EPS, stride, w->shape[2] / 2, VD_ACT_SILU,
                            0.f, &idx);
    if (rc) return rc;
    c.plate.conv_idx.push_back({pre, idx});
    return VD_OK;
}

// model.0 (3x3, stride 2, pad 1, 3 -> 16, BN + SiLU) over the space-to-depth canvas
// X'[Y][X][(py*2+px)*4 + c] = x[2Y+py-1][2X+px-1][c] (the face stem's form, pre.hip):
// a 2x2, stride-1, pad-0 conv with 16 input channels, W'[n][(py*2+px)*4+c][ta][tb] =
// W[n][c][2ta+py][2tb+px] (zero where 2ta+py or 2tb+px is 3, and for the 4th channel
// of each sub-pixel). Same 27 products per output; the canvas is 8 B per pixel
// instead of 16 (cpad 8).
int yconv_s2d(Ctx& c, const WMap& W, const std::string& pre) {
    const HT* w = find_t(W, pre + ".conv.weight");
    const HT* g = find_t(W, pre + ".bn.weight");
    const HT* b = find_t(W, pre + ".bn.bias");
    const HT* m = find_t(W, pre + ".bn.running_mean");
    const HT* v = find_t(W, pre + ".bn.running_var");
    if (!w || w->shape.size() != 4 || w->shape[1] != 3 || w->shape[2] != 3 || w->shape[3] != 3)
        return vd_set_error(VD_ERR_WEIGHTS, "missing/bad %s.conv.weight", pre.c_str());
    if (!g || !b || !m || !v) return vd_set_error(VD_ERR_WEIGHTS, "missing BatchNorm tensors under %s.bn", pre.c_str());
    Conv cv{};
    cv.cout = w->shape[0]; cv.cin = 16; cv.kh = 2; cv.kw = 2;
    cv.stride = 1; cv.pad = 0; cv.act = VD_ACT_SILU; cv.slope = 0.f;
    std::vector<float> wt((size_t)cv.cout * 16 * 4, 0.f), sc(cv.cout), sh(cv.cout);
    for (int n = 0; n < cv.cout; ++n) {
        for (int ta = 0; ta < 2; ++ta)
            for (int tb = 0; tb < 2; ++tb)
                for (int py = 0; py < 2; ++py)
                    for (int px = 0; px < 2; ++px)
                        for (int ch = 0; ch < 3; ++ch) {
                            const int dy = 2 * ta + py, dx = 2 * tb + px;
                            if (dy > 2 || dx > 2) continue;
                            wt[(((size_t)n * 16 + (py * 2 + px) * 4 + ch) * 2 + ta) * 2 + tb] =
                                w->data[(((size_t)n * 3 + ch) * 3 + dy) * 3 + dx];
                        }
        const float alpha = g->data[n] / std::sqrt(v->data[n] + YOLO_BN_EPS);
        // fp32 plan: the canvas holds the integer pixel values (exact in fp16), the
        // preprocessing's / 255 moves into the BN scale
        sc[n] = c.f32 ? alpha / 255.f : alpha;
        sh[n] = b->data[n] - m->data[n] * alpha;
    }
    int rc = c.upload_conv(cv, wt, sc, sh);
    if (rc) return rc;
    cv.flops_per_px = 2.0 * cv.cout * 3 * 9;   // algorithmic work of the original 3x3 conv
    c.convs.push_back(cv);
    c.plate.conv_idx.push_back({pre, (int)c.convs.size() - 1});
    return VD_OK;
}

// Two Conv+BN+SiLU with the same input fused along Cout (Detect cv2.i.0 | cv3.i.0).
int yconv_pair(Ctx& c, const WMap& W, const std::string& a, const std::string& b, const std::string& name) {
    Conv cv{};
    std::vector<float> wall, sc, sh;
    for (const std::string& pre : {a, b}) {
        const HT* w = find_t(W, pre + ".conv.weight");
        const HT* g = find_t(W, pre + ".bn.weight");
        const HT* bb = find_t(W, pre + ".bn.bias");
        const HT* m = find_t(W, pre + ".bn.running_mean");
        const HT* v = find_t(W, pre + ".bn.running_var");
        if (!w || !g || !bb || !m || !v) return vd_set_error(VD_ERR_WEIGHTS, "missing tensors under %s", pre.c_str());
        if (cv.cout == 0) { cv.cin = w->shape[1]; cv.kh = w->shape[2]; cv.kw = w->shape[3]; }
        wall.insert(wall.end(), w->data.begin(), w->data.end());
        for (int n = 0; n < w->shape[0]; ++n) {
            const float alpha = g->data[n] / std::sqrt(v->data[n] + YOLO_BN_EPS);
            sc.push_back(alpha);
            sh.push_back(bb->data[n] - m->data[n] * alpha);
        }
        cv.cout += w->shape[0];
    }
    cv.stride = 1; cv.pad = cv.kh / 2; cv.act = VD_ACT_SILU;
    int rc = c.upload_conv(cv, wall, sc, sh);
    if (rc) return rc;
    c.convs.push_back(cv);
    c.plate.conv_idx.push_back({name, (int)c.convs.size() - 1});
    return VD_OK;
}

// The Detect head's cv2.i.1 and cv3.i.1 (3x3, 64 -> 64 each, on the two halves of det0.i's
// output) as one grouped conv: output rows [0, 64) read input channels [0, 64), rows
// [64, 128) channels [64, 128) (fp32 plan: conv_x6_halo_kernel, one 64-wide N tile per
// group). Same products per output as the two convs: bit-identical.
int yconv_group(Ctx& c, const WMap& W, const std::string& a, const std::string& b, const std::string& name) {
    int rc = yconv_pair(c, W, a, b, name);
    if (rc) return rc;
    Conv& cv = c.convs[conv_of(c.plate, name)];
    if (cv.cin != 64 || cv.cout != 128) return vd_set_error(VD_ERR_WEIGHTS, "unsupported Detect head widths");
    cv.grp_co = 64;
    cv.grp_ci = 64;
    return VD_OK;
}

int yhead(Ctx& c, const WMap& W, const std::string& pre, const std::string& name) {
    int idx;
    int rc = c.make_conv_cat(W, {pre + ".weight"}, {pre + ".bias"}, VD_ACT_NONE, &idx);
    if (rc) return rc;
    c.plate.conv_idx.push_back({name, idx});
    return VD_OK;
}

int c2f_convs(Ctx& c, const WMap& W, const std::string& pre, int n) {
    int rc;
    if ((rc = yconv(c, W, pre + ".cv1", 1))) return rc;
    if ((rc = yconv(c, W, pre + ".cv2", 1))) return rc;
    for (int i = 0; i < n; ++i) {
        if ((rc = yconv(c, W, pre + ".m." + std::to_string(i) + ".cv1", 1))) return rc;
        if ((rc = yconv(c, W, pre + ".m." + std::to_string(i) + ".cv2", 1))) return rc;
    }
    return VD_OK;
}

struct Planner {
    Ctx& c;
    Net& net;
    int ch, cw;
    int rc = VD_OK;
    Act buf(const std::string& n) {
        const Act* b = find_buf(c.plate, n);
        Act a = *b;
        int div = 1;
        for (const Buf& k : kBufs)
            if (n == k.name) div = k.div;
        a.h = ch / div;
        a.w = cw / div;
        return a;
    }
    void conv(const std::string& name, const Act& x, int xcoff, Act y, int ycoff, const Act* res = nullptr,
              int rcoff = 0) {
        if (rc) return;
        const int ci = conv_of(c.plate, name);
        if (ci < 0) { rc = vd_set_error(VD_ERR_STATE, "plate conv %s not built", name.c_str()); return; }
        rc = c.add_conv(net, ci, x, xcoff, y, ycoff, res, rcoff, res ? VD_RES_POST_ACT : VD_RES_NONE, 0);
    }
    // C2f: cv1 -> [y0|y1] at buf[0:2c); bottleneck i reads slice (1+i), writes slice (2+i);
    // cv2 over the (2+n)c concat -> out.
    void c2f(const std::string& pre, int n, bool shortcut, const Act& x, int xcoff, const std::string& cb,
             const std::string& tb, Act out, int ocoff) {
        Act C = buf(cb), T = buf(tb);
        const int cc = c.convs[conv_of(c.plate, pre + ".m.0.cv1")].cin;
        conv(pre + ".cv1", x, xcoff, C, 0);
        for (int i = 0; i < n; ++i) {
            const std::string m = pre + ".m." + std::to_string(i);
            conv(m + ".cv1", C, (1 + i) * cc, T, 0);
            conv(m + ".cv2", T, 0, C, (2 + i) * cc, shortcut ? &C : nullptr, (1 + i) * cc);
        }
        conv(pre + ".cv2", C, 0, out, ocoff);
    }
    void pool(const Act& x, int xcoff, Act y, int ycoff, int ch_) {
        if (rc) return;
        Op op;
        op.kind = OP_MAXPOOL;
        op.x = x; op.xcoff = xcoff; op.y = y; op.ycoff = ycoff; op.ch = ch_; op.k = 5; op.s = 1; op.p = 2;
        net.ops.push_back(op);
    }
    void up(const Act& x, int xcoff, Act y, int ycoff, int ch_) {
        if (rc) return;
        Op op;
        op.kind = OP_UPSAMPLE;
        op.x = x; op.xcoff = xcoff; op.y = y; op.ycoff = ycoff; op.ch = ch_;
        net.ops.push_back(op);
    }
};

int build_plan(Ctx& c, int ch, int cw, Net& net) {
    PlateNet& P = c.plate;
    Planner p{c, net, ch, cw};
    net.amax = c.amax_region(1);
    net.amax_bytes = net.amax ? c.amax_region_bytes() : 0;
    Act in = P.input;
    in.h = P.s2d ? ch / 2 + 1 : ch;
    in.w = P.s2d ? cw / 2 + 1 : cw;
    p.conv("model.0", in, 0, p.buf("A0"), 0);
    p.conv("model.1", p.buf("A0"), 0, p.buf("A1"), 0);
    p.c2f("model.2", 1, true, p.buf("A1"), 0, "C2", "T2", p.buf("A2"), 0);
    p.conv("model.3", p.buf("A2"), 0, p.buf("A3"), 0);
    p.c2f("model.4", 2, true, p.buf("A3"), 0, "C4", "T4", p.buf("cat14"), 128);          // P3 route -> cat14[128:192)
    p.conv("model.5", p.buf("cat14"), 128, p.buf("A5"), 0);
    p.c2f("model.6", 2, true, p.buf("A5"), 0, "C6", "T6", p.buf("cat11"), 256);         // P4 route -> cat11[256:384)
    p.conv("model.7", p.buf("cat11"), 256, p.buf("A7"), 0);
    p.c2f("model.8", 1, true, p.buf("A7"), 0, "C8", "T8", p.buf("A8"), 0);
    // SPPF: cv1 -> S9[0:128), 3x maxpool5 -> S9[128:256),[256:384),[384:512), cv2 -> cat20[128:384)
    p.conv("model.9.cv1", p.buf("A8"), 0, p.buf("S9"), 0);
    p.pool(p.buf("S9"), 0, p.buf("S9"), 128, 128);
    p.pool(p.buf("S9"), 128, p.buf("S9"), 256, 128);
    p.pool(p.buf("S9"), 256, p.buf("S9"), 384, 128);
    p.conv("model.9.cv2", p.buf("S9"), 0, p.buf("cat20"), 128);
    p.up(p.buf("cat20"), 128, p.buf("cat11"), 0, 256);                                   // 10,11
    p.c2f("model.12", 1, false, p.buf("cat11"), 0, "C12", "T12", p.buf("cat17"), 64);   // -> cat17[64:192)
    p.up(p.buf("cat17"), 64, p.buf("cat14"), 0, 128);                                    // 13,14
    // Detect level i (model.22 cv2.i / cv3.i on P3 / P4 / P5, combine_detect.py:872 via
    // ultralytics [ext]); each level reads only its P buffer and writes its own head slice
    const char* lv[3] = {"P3", "P4", "P5"};
    auto detect = [&](int i) {
        const std::string I = std::to_string(i);
        Act d0 = p.buf("D0_" + I), d1 = p.buf("D1_" + I);
        Act hd = P.head[i];
        hd.h = ch / (8 << i); hd.w = cw / (8 << i);
        p.conv("det0." + I, p.buf(lv[i]), 0, d0, 0);
        if (conv_of(P, "det1." + I) >= 0 && hd.w <= 126 && c.tune.x6_halo) {   // the halo tile's width limit
            p.conv("det1." + I, d0, 0, d1, 0);
        } else {
            p.conv("model.22.cv2." + I + ".1", d0, 0, d1, 0);
            p.conv("model.22.cv3." + I + ".1", d0, 64, d1, 64);
        }
        p.conv("box." + I, d1, 0, hd, 0);
        p.conv("cls." + I, d1, 64, hd, 64);
    };
    // option plate_detect_early (default 1): each Detect level right after its P level is
    // produced, so the heavy level-0 head (P3, 80 x 48) overlaps the face net instead of
    // ending the plate branch -- the branch's last launches are then the small 20 x 12 tail
    const bool early = c.tune.plate_detect_early != 0;
    p.c2f("model.15", 1, false, p.buf("cat14"), 0, "C15", "T15", p.buf("P3"), 0);
    if (early) detect(0);
    p.conv("model.16", p.buf("P3"), 0, p.buf("cat17"), 0);                               // 16,17
    p.c2f("model.18", 1, false, p.buf("cat17"), 0, "C18", "T18", p.buf("P4"), 0);
    if (early) detect(1);
    p.conv("model.19", p.buf("P4"), 0, p.buf("cat20"), 0);                               // 19,20
    p.c2f("model.21", 1, false, p.buf("cat20"), 0, "C21", "T21", p.buf("P5"), 0);
    for (int i = early ? 2 : 0; i < 3; ++i) detect(i);
    return p.rc;
}
}  // namespace

int vd_build_plate(Ctx& c, const WMap& W) {
    PlateNet& P = c.plate;
    P.nc = c.cfg.plate_nc;
    P.imgsz = c.cfg.plate_imgsz > 0 ? c.cfg.plate_imgsz : 640;
    if (P.imgsz % 32) return vd_set_error(VD_ERR_ARG, "plate_imgsz must be a multiple of 32");
    const HT* cls0 = find_t(W, "model.22.cv3.0.2.weight");
    if (!cls0) return vd_set_error(VD_ERR_WEIGHTS, "missing model.22.cv3.0.2.weight (YOLOv8 Detect head)");
    if (cls0->shape[0] != P.nc)
        return vd_set_error(VD_ERR_WEIGHTS, "plate weights have %d classes, cfg.plate_nc = %d", cls0->shape[0], P.nc);
    int rc;
    static const int strides[] = {2, 2, 1, 2, 1, 2, 1, 2, 1};
    // bf16 / fp32 (fp16 pairs): the letterbox writes the stem input in space-to-depth form
    // (option plate_s2d=0: off); fp32 as integer pixel values in f32 (exact in fp16),
    // model.0 then on one A plane (x_exact) with the / 255 in its BN scale
    P.s2d = c.tune.plate_s2d && (!c.f32 || (c.tune.f32_split == 2 && c.tune.plate_s2d32));
    if (P.s2d && (rc = yconv_s2d(c, W, "model.0"))) return rc;
    for (int i : {0, 1, 3, 5, 7}) {
        if (i == 0 && P.s2d) continue;
        if ((rc = yconv(c, W, "model." + std::to_string(i), strides[i]))) return rc;
    }
    for (int i : {16, 19}) if ((rc = yconv(c, W, "model." + std::to_string(i), 2))) return rc;
    if ((rc = c2f_convs(c, W, "model.2", 1))) return rc;
    if ((rc = c2f_convs(c, W, "model.4", 2))) return rc;
    if ((rc = c2f_convs(c, W, "model.6", 2))) return rc;
    if ((rc = c2f_convs(c, W, "model.8", 1))) return rc;
    if ((rc = yconv(c, W, "model.9.cv1", 1))) return rc;
    if ((rc = yconv(c, W, "model.9.cv2", 1))) return rc;
    for (int i : {12, 15, 18, 21}) if ((rc = c2f_convs(c, W, "model." + std::to_string(i), 1))) return rc;
    for (int i = 0; i < 3; ++i) {
        const std::string I = std::to_string(i);
        if ((rc = yconv_pair(c, W, "model.22.cv2." + I + ".0", "model.22.cv3." + I + ".0", "det0." + I))) return rc;
        if ((rc = yconv(c, W, "model.22.cv2." + I + ".1", 1))) return rc;
        if ((rc = yconv(c, W, "model.22.cv3." + I + ".1", 1))) return rc;
        if (c.f32 && c.tune.f32_split == 2 && c.tune.det_group &&
            (rc = yconv_group(c, W, "model.22.cv2." + I + ".1", "model.22.cv3." + I + ".1", "det1." + I)))
            return rc;
        if ((rc = yhead(c, W, "model.22.cv2." + I + ".2", "box." + I))) return rc;
        if ((rc = yhead(c, W, "model.22.cv3." + I + ".2", "cls." + I))) return rc;
        if (c.convs[conv_of(P, "box." + I)].cout != 64 || c.convs[conv_of(P, "det0." + I)].cout != 128)
            return vd_set_error(VD_ERR_WEIGHTS, "unsupported Detect head widths (expect reg_max 16, c2 = c3 = 64)");
    }
    // buffers for the imgsz x imgsz canvas
    const int cpad = c.f32 ? 4 : 8;
    c.amax_begin(1);
    if (P.s2d) rc = c.act(P.input, P.imgsz / 2 + 1, P.imgsz / 2 + 1, 16);   // fp32: f32 (conv_x6 reads f32 A)
    else rc = c.act(P.input, P.imgsz, P.imgsz, cpad);
    if (rc) return rc;
    P.input.amax = nullptr;            // letterboxed canvas / 255: in [0, 1]
    P.input.bound = 1.f;
    if (P.s2d && c.f32) {              // fp32 s2d canvas: integer pixel values 0..255
        P.input.bound = 255.f;
        P.input.exact16 = true;
    }
    for (const Buf& b : kBufs) {
        Act a;
        if ((rc = c.act(a, P.imgsz / b.div, P.imgsz / b.div, b.c))) return rc;
        P.bufs.push_back({b.name, a});
    }
    P.hstride = (64 + P.nc + 7) / 8 * 8;   // 8-channel multiple: 16-B vector epilogues for the box head
    P.A_max = 0;
    for (int i = 0; i < 3; ++i) {
        const int s = P.imgsz / (8 << i);
        if ((rc = c.act(P.head[i], s, s, P.hstride, true))) return rc;
        P.A_max += s * s;
    }
    const int kcap = c.cfg.plate_max_det > 0 ? std::min(P.A_max, c.cfg.plate_max_det) : P.A_max;
    if ((rc = vd_alloc_post(c, P.post, P.A_max, kcap))) return rc;
    P.loaded = true;
    return VD_OK;
}

// ultralytics LetterBox(imgsz, auto=True, stride=32) geometry [ext] (oracle/letterbox.py)
static void yolo_geometry(int ih, int iw, int imgsz, int* nw, int* nh, int* top, int* left, int* oh, int* ow) {
    const double r = std::min((double)imgsz / ih, (double)imgsz / iw);
    *nw = (int)std::nearbyint(iw * r);
    *nh = (int)std::nearbyint(ih * r);
    double dw = (imgsz - *nw) % 32, dh = (imgsz - *nh) % 32;
    dw /= 2;
    dh /= 2;
    *top = (int)std::nearbyint(dh - 0.1);
    const int bottom = (int)std::nearbyint(dh + 0.1);
    *left = (int)std::nearbyint(dw - 0.1);
    const int right = (int)std::nearbyint(dw + 0.1);
    *oh = *nh + *top + bottom;
    *ow = *nw + *left + right;
}

int vd_plate_letterbox_args(Ctx& c, const uint8_t* d, int n, int h, int w, size_t pitch, LetterboxArgs* out) {
    PlateNet& P = c.plate;
    int nw, nh, top, left, oh, ow;
    yolo_geometry(h, w, P.imgsz, &nw, &nh, &top, &left, &oh, &ow);
    if (oh > P.imgsz || ow > P.imgsz || oh % 32 || ow % 32)
        return vd_set_error(VD_ERR_ARG, "plate canvas %dx%d unsupported", ow, oh);
    LetterboxArgs a{};
    a.src = d; a.n = n; a.ih = h; a.iw = w; a.pitch = pitch;
    a.oh = oh; a.ow = ow; a.nh = nh; a.nw = nw; a.top = top; a.left = left;
    vd_resize_mode(h, w, nh, nw, &a.mode, &a.scale_x, &a.scale_y);
    a.pad_value = 114.f;
    a.mean[0] = a.mean[1] = a.mean[2] = 0.f;
    a.div = P.s2d && c.f32 ? 1.f : 255.f;   // fp32 s2d: integers, / 255 in model.0's BN scale
    a.flip = 1;   // im[..., ::-1]: the RGB frames are treated as BGR
    a.out = P.input.p; a.cpad = P.input.c; a.out_f32 = c.f32 ? 1 : 0; a.out_f16 = c.f16 ? 1 : 0;
    a.s2d = P.s2d ? 1 : 0;
    *out = a;
    return VD_OK;
}

int vd_plate_forward(Ctx& c, const uint8_t* d, int n, int h, int w, size_t pitch, bool letterboxed) {
    PlateNet& P = c.plate;
    LetterboxArgs a;
    int rc0 = vd_plate_letterbox_args(c, d, n, h, w, pitch, &a);
    if (rc0) return rc0;
    const int oh = a.oh, ow = a.ow;
    if (!letterboxed) {
        const double obytes =
            P.s2d ? (double)(oh / 2 + 1) * (ow / 2 + 1) * (c.f32 ? 64 : 32) : (double)oh * ow * a.cpad * (c.f32 ? 4 : 2);
        c.t_begin(2, (double)n * (a.nh * (double)w * 3 + obytes));
        hipError_t e = vd_launch_letterbox(a, c.stream);
        c.t_end();
        if (e != hipSuccess) return vd_set_error(VD_ERR_HIP, "plate letterbox: %s", hipGetErrorString(e));
    }
    const long long key = ((long long)oh << 32) | ow;
    Net* net = nullptr;
    for (auto& pl : P.plans)
        if (pl.first == key) net = &pl.second;
    if (!net) {
        P.plans.push_back({key, Net{}});
        P.plans.back().second.conv_fam = 5;
        net = &P.plans.back().second;
        int rc = build_plan(c, oh, ow, *net);
        if (rc) { P.plans.pop_back(); return rc; }
    }
    P.ch = oh; P.cw = ow;
    P.A = 0;
    for (int i = 0; i < 3; ++i) {
        P.lh[i] = oh / (8 << i);
        P.lw[i] = ow / (8 << i);
        P.loff[i] = P.A;
        P.A += P.lh[i] * P.lw[i];
    }
    return c.run_net(*net, n);
}

int vd_plate_post(Ctx& c, int n, int img_h, int img_w, const BoxTargets& t) {
    PlateNet& P = c.plate;
    PostArgs p{};
    p.mode = POST_YOLO;
    for (int l = 0; l < 3; ++l) {
        p.heads[l] = (const float*)P.head[l].p;
        p.lh[l] = P.lh[l]; p.lw[l] = P.lw[l]; p.loff[l] = P.loff[l];
        p.strides[l] = 8 << l;
    }
    p.hstride = P.hstride;
    p.A = P.A; p.B = n; p.nc = P.nc;
    p.conf = c.cfg.plate_conf; p.iou = c.cfg.plate_iou; p.max_det = c.cfg.plate_max_det; p.max_wh = MAX_WH;
    p.cand_keys = P.post.keys; p.cand_count = P.post.count;
    p.scratch_box = P.post.box; p.scratch_cls = P.post.cls; p.scratch_nbox = P.post.nbox;
    p.scratch_area = P.post.area; p.scratch_keys = P.post.sort; p.scratch_supp = P.post.supp;
    p.sort_cap = P.post.sort_cap;
    p.img_h = img_h; p.img_w = img_w;
    // scale_boxes(img1_shape=(ch, cw), boxes, img0_shape=(h, w)) [ext], Python floats
    const double gain = std::min((double)P.ch / img_h, (double)P.cw / img_w);
    p.padx = (int)std::nearbyint((P.cw - img_w * gain) / 2 - 0.1);
    p.pady = (int)std::nearbyint((P.ch - img_h * gain) / 2 - 0.1);
    p.inv_gain = 1.0f / (float)gain;   // torch divides a tensor by a Python scalar as x * (1/b)
    p.cap = t.cap; p.out_count = t.count; p.out_xyxy = t.xyxy; p.out_xyxy_f = t.xyxy_f;
    p.out_score = t.score; p.out_label = t.label;
    vd_post_keep_args(P.post, p, n);
    c.t_begin(3, (double)n * P.A * P.hstride * 4);
    hipError_t e = vd_launch_post(p, c.stream);
    c.t_end();
    if (e != hipSuccess) return vd_set_error(VD_ERR_HIP, "plate post: %s", hipGetErrorString(e));
    return VD_OK;
}

extern "C" int vdt_plate_raw(vd_ctx* h, const uint8_t* frames, int n, int fh, int fw, size_t pitch, int where,
                             float* out, int* anchors) {
    Ctx* ctx = (Ctx*)h;
    if (!ctx) return vd_set_error(VD_ERR_ARG, "null context");
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (hipSetDevice(ctx->device) != hipSuccess) return vd_set_error(VD_ERR_HIP, "hipSetDevice");
    if (!ctx->plate.loaded) return vd_set_error(VD_ERR_STATE, "plate weights not loaded");
    int rc = ctx->check_frames(n, fh, fw, pitch);
    if (rc) return rc;
    const uint8_t* d = ctx->frames_to_device(frames, n, fh, pitch, where, &rc);
    if (rc) return rc;
    if ((rc = vd_plate_forward(*ctx, d, n, fh, fw, pitch))) return rc;
    VD_CHECK_HIP(hipStreamSynchronize(ctx->stream));
    PlateNet& P = ctx->plate;
    if (anchors) *anchors = P.A;
    if (!out) return VD_OK;
    // raw head tensors -> [n][64 + nc][A] (box DFL logits, class logits), anchor order level/y/x
    const int C = 64 + P.nc;
    for (int l = 0; l < 3; ++l) {
        const Act& hd = P.head[l];
        const size_t px = (size_t)P.lh[l] * P.lw[l];
        std::vector<float> buf((size_t)n * px * P.hstride);
        VD_CHECK_HIP(hipMemcpy(buf.data(), hd.p, buf.size() * 4, hipMemcpyDeviceToHost));
        for (int b = 0; b < n; ++b)
            for (size_t q = 0; q < px; ++q)
                for (int ch = 0; ch < C; ++ch)
                    out[((size_t)b * C + ch) * P.A + P.loff[l] + q] = buf[((size_t)b * px + q) * P.hstride + ch];
    }
    return VD_OK;
}
