// face_net.cpp — RetinaFace-ResNet50 plan (cfg_re50) on the conv/pool kernels.
//
// Module tree = reference state_dict keys (detect_face/retinaface.py:53-92):
//   body.*            torchvision resnet50 up to layer4 [ext] (v1.5, stride on the 3x3)
//   fpn.output{1,2,3} 1x1 conv+BN+ReLU (layers.py:72-74; leaky=0 as out=256>64, :71)
//   fpn.merge{1,2}    3x3 conv+BN+ReLU, input = lateral + nearest-2x(upper) (:100-110)
//   ssh{1,2,3}        SSH (layers.py:37-66): concat of three branches, then ReLU
//   {Bbox,Class,Landmark}Head.{l}.conv1x1   1x1 heads (retinaface.py:13-51)
// Fusions: BN (eval) + activation + residual in every conv epilogue; the FPN
// upsample-add is the lateral conv's epilogue (nearest-2x residual); the SSH
// concat is convs writing channel slices of one buffer with the post-concat ReLU
// applied per slice (ReLU SSH: [t5 | c3 | c5 | c7], conv5X5_1 and conv3X3 as one
// 192-channel conv, the heads reading [c3 | c5 | c7]); the three heads of a level
// are one 256->32 conv (channels 0-7 bbox, 8-11 class, 12-31 landm).
#include "nets.h"
#include "vd_math.h"

#include <cmath>
#include <cstdlib>
#include <string>
#include <vector>

namespace {
constexpr float BN_EPS = 1e-5f;   // nn.BatchNorm2d default (torchvision + layers.py)

int conv_bn(Ctx& c, const WMap& W, const std::string& conv, const std::string& bn, int stride, int pad, int act,
            int* idx) {
    return c.make_conv_bn(W, conv, bn, BN_EPS, stride, pad, act, 0.f, idx);
}

// The stem conv1 (7x7, stride 2, pad 3, 3 -> 64) rewritten over the space-to-depth
// input X'[Y][X][(py*2+px)*4 + c] = x[2Y+py-1][2X+px-1][c]: a 4x4, stride-1, pad-1
// conv with 16 input channels, W'[n][(py*2+px)*4+c][ta][tb] = W[n][c][2ta+py][2tb+px]
// (zero where 2ta+py or 2tb+px is 7, and for the 4th channel of each sub-pixel).
// Same products and the same sum (K 147 real terms of 256 instead of 147 of 448).
int stem_s2d(Ctx& c, const WMap& W, int* idx) {
    const HT* w = find_t(W, "body.conv1.weight");
    const HT* g = find_t(W, "body.bn1.weight");
    const HT* b = find_t(W, "body.bn1.bias");
    const HT* m = find_t(W, "body.bn1.running_mean");
    const HT* v = find_t(W, "body.bn1.running_var");
    if (!w || w->shape.size() != 4 || w->shape[1] != 3 || w->shape[2] != 7 || w->shape[3] != 7)
        return vd_set_error(VD_ERR_WEIGHTS, "missing/bad body.conv1.weight");
    if (!g || !b || !m || !v) return vd_set_error(VD_ERR_WEIGHTS, "missing BatchNorm tensors under body.bn1");
    Conv cv{};
    cv.cout = w->shape[0]; cv.cin = 16; cv.kh = 4; cv.kw = 4;
    cv.stride = 1; cv.pad = 1; cv.act = VD_ACT_RELU; cv.slope = 0.f;
    std::vector<float> wt((size_t)cv.cout * 16 * 16, 0.f), sc(cv.cout), sh(cv.cout);
    for (int n = 0; n < cv.cout; ++n) {
        for (int ta = 0; ta < 4; ++ta)
            for (int tb = 0; tb < 4; ++tb)
                for (int py = 0; py < 2; ++py)
                    for (int px = 0; px < 2; ++px)
                        for (int ch = 0; ch < 3; ++ch) {
                            const int dy = 2 * ta + py, dx = 2 * tb + px;
                            if (dy > 6 || dx > 6) continue;
                            const int ci = (py * 2 + px) * 4 + ch;
                            wt[(((size_t)n * 16 + ci) * 4 + ta) * 4 + tb] = w->data[(((size_t)n * 3 + ch) * 7 + dy) * 7 + dx];
                        }
        const float alpha = g->data[n] / std::sqrt(v->data[n] + BN_EPS);
        sc[n] = alpha;
        sh[n] = b->data[n] - m->data[n] * alpha;
    }
    int rc = c.upload_conv(cv, wt, sc, sh);
    if (rc) return rc;
    cv.flops_per_px = 2.0 * cv.cout * 3 * 49;   // algorithmic work of the original 7x7 conv
    c.convs.push_back(cv);
    *idx = (int)c.convs.size() - 1;
    return VD_OK;
}
// MobileNetV1-0.25 body (detect_face/nets/mobilenet025.py:21-48, cfg_mnet
// return_layers stage1/2/3 -> 64/128/256 channels at strides 8/16/32): conv_bn(3, 8, 2)
// then conv_dw blocks = depthwise 3x3 (+BN+LeakyReLU 0.1, dwconv.hip) and pointwise
// 1x1 (+BN+LeakyReLU 0.1, the streaming 1x1 kernel). Keys: body.stageS.I.{0,1}
// (conv_bn) and body.stageS.I.{0,1,3,4} (conv_dw: dw conv, bn, pw conv, bn).
int build_mnet_body(Ctx& c, const WMap& W, FaceNet& F, Act feats[3]) {
    constexpr float SLOPE = 0.1f;
    int rc, ci;
    const HT* w0 = find_t(W, "body.stage1.0.0.weight");
    if (!w0 || w0->shape.size() != 4) return vd_set_error(VD_ERR_WEIGHTS, "missing body.stage1.0.0.weight");
    if ((rc = c.make_conv_bn(W, "body.stage1.0.0.weight", "body.stage1.0.1", BN_EPS, 2, 1, VD_ACT_LEAKY, SLOPE, &ci)))
        return rc;
    Act x;
    if ((rc = c.act(x, (F.input.h - 1) / 2 + 1, (F.input.w - 1) / 2 + 1, c.convs[ci].cout))) return rc;
    if ((rc = c.add_conv(F.net, ci, F.input, 0, x, 0))) return rc;
    F.net.stage_end[0] = (int)F.net.ops.size();
    // (stage, number of modules, strides of the conv_dw modules)
    const int nmod[3] = {6, 6, 2};
    for (int st = 0; st < 3; ++st) {
        for (int i = (st == 0 ? 1 : 0); i < nmod[st]; ++i) {
            const std::string p = "body.stage" + std::to_string(st + 1) + "." + std::to_string(i);
            const HT* pw = find_t(W, p + ".3.weight");
            if (!pw || pw->shape.size() != 4) return vd_set_error(VD_ERR_WEIGHTS, "missing %s.3.weight", p.c_str());
            // stride 2 on the first module of stage2/3 and on stage1 modules 2 and 4 (:29-33)
            const int s = (st == 0 && (i == 2 || i == 4)) || (st > 0 && i == 0) ? 2 : 1;
            int di, pi;
            if ((rc = c.make_dwconv_bn(W, p + ".0.weight", p + ".1", BN_EPS, s, VD_ACT_LEAKY, SLOPE, &di))) return rc;
            if ((rc = c.make_conv_bn(W, p + ".3.weight", p + ".4", BN_EPS, 1, 0, VD_ACT_LEAKY, SLOPE, &pi))) return rc;
            Act t, y;
            if ((rc = c.act(t, (x.h - 1) / s + 1, (x.w - 1) / s + 1, x.c))) return rc;
            if ((rc = c.add_dwconv(F.net, di, x, t))) return rc;
            if ((rc = c.act(y, t.h, t.w, c.convs[pi].cout))) return rc;
            if ((rc = c.add_conv(F.net, pi, t, 0, y, 0))) return rc;
            x = y;
        }
        feats[st] = x;
        F.net.stage_end[st + 1] = (int)F.net.ops.size();
    }
    F.net.stage_end[4] = (int)F.net.ops.size();
    return VD_OK;
}
}  // namespace

int vd_build_face(Ctx& c, const WMap& W) {
    FaceNet& F = c.face;
    for (hipEvent_t ev : c.lane_ev)   // a previous load's lane events (face_lanes re-creates them)
        if (ev) hipEventDestroy(ev);
    c.lane_ev.clear();
    F.in_h = c.cfg.input_h;
    F.in_w = c.cfg.input_w;
    const int H = F.in_h, Wd = F.in_w;
    const int cpad = c.f32 ? 4 : 8;
    int rc;
    F.mnet = find_t(W, "body.stage1.0.0.weight") != nullptr;   // cfg_mnet (face.py:35, retinaface.py:60)
    // fp32 plan (fp16 pairs): the fused stem + pool on an fp16 space-to-depth canvas
    const bool s2d32 = c.f32 && c.tune.f32_split == 2 && c.tune.stem_pool &&
                       vd_stem_pool_ok(H / 2 + 1, Wd / 2 + 1, H / 4, Wd / 4);
    F.s2d = (!c.f32 || s2d32) && !F.mnet && H % 2 == 0 && Wd % 2 == 0;   // bf16 / fp16 / fp32 pairs
    c.amax_begin(0);
    if (F.s2d) rc = c.act(F.input, H / 2 + 1, Wd / 2 + 1, 16, false, c.f32);
    else rc = c.act(F.input, H, Wd, cpad);
    if (rc) return rc;
    F.input.amax = nullptr;            // letterboxed canvas: |pixel - mean| <= 255
    F.input.bound = 255.f;
    F.input.exact16 = true;            // integers (pixel, means 104/117/123, pad 128)

    Act feats[3];
    if (F.mnet) {
        if ((rc = build_mnet_body(c, W, F, feats))) return rc;
    } else {
    // ---- stem: conv1 7x7/2 + bn1 + relu, maxpool 3x3/2 pad 1 ----
    int ci;
    if (F.s2d) rc = stem_s2d(c, W, &ci);
    else rc = conv_bn(c, W, "body.conv1.weight", "body.bn1", 2, 3, VD_ACT_RELU, &ci);
    if (rc) return rc;
    Act stem, pool;
    if ((rc = c.act(pool, H / 4, Wd / 4, 64))) return rc;
    if (F.s2d && c.tune.stem_pool && vd_stem_pool_ok(F.input.h, F.input.w, pool.h, pool.w)) {
        // conv1 + bn1 + relu + maxpool in one kernel (stem.hip): the stem map stays on chip
        if ((rc = c.add_stem_pool(F.net, ci, F.input, pool))) return rc;
    } else {
        if ((rc = c.act(stem, H / 2, Wd / 2, 64))) return rc;
        if ((rc = c.add_conv(F.net, ci, F.input, 0, stem, 0))) return rc;
        Op op;
        op.kind = OP_MAXPOOL;
        op.x = stem; op.y = pool; op.ch = 64; op.k = 3; op.s = 2; op.p = 1;
        F.net.ops.push_back(op);
    }
    F.net.stage_end[0] = (int)F.net.ops.size();

    // ---- layer1..4 (Bottleneck x [3,4,6,3]) ----
    Act x = pool;
    const int planes_l[4] = {64, 128, 256, 512}, blocks_l[4] = {3, 4, 6, 3}, stride_l[4] = {1, 2, 2, 2};
    for (int li = 0; li < 4; ++li) {
        const int planes = planes_l[li];
        const size_t layer_begin = F.net.ops.size();
        for (int bi = 0; bi < blocks_l[li]; ++bi) {
            const std::string pre = "body.layer" + std::to_string(li + 1) + "." + std::to_string(bi);
            const int s = bi == 0 ? stride_l[li] : 1;
            int c1, c2, c3, cd = -1;
            if ((rc = conv_bn(c, W, pre + ".conv1.weight", pre + ".bn1", 1, 0, VD_ACT_RELU, &c1))) return rc;
            if ((rc = conv_bn(c, W, pre + ".conv2.weight", pre + ".bn2", s, 1, VD_ACT_RELU, &c2))) return rc;
            if ((rc = conv_bn(c, W, pre + ".conv3.weight", pre + ".bn3", 1, 0, VD_ACT_RELU, &c3))) return rc;
            const bool has_ds = find_t(W, pre + ".downsample.0.weight") != nullptr;
            if (has_ds && (rc = conv_bn(c, W, pre + ".downsample.0.weight", pre + ".downsample.1", s, 0, VD_ACT_NONE, &cd)))
                return rc;
            if (!has_ds && (s != 1 || x.c != planes * 4))
                return vd_set_error(VD_ERR_WEIGHTS, "%s: missing downsample", pre.c_str());
            const int oh = x.h / s, ow = x.w / s;
            Act t1, t2, out, ds;
            if (s == 1 && c.block_ok(c1, c2, c3, cd, x)) {
                // the whole bottleneck in one kernel (block.hip): t1/t2 stay in LDS
                int bk;
                if ((rc = c.act(out, oh, ow, planes * 4))) return rc;
                if ((rc = c.make_block(c1, c2, c3, cd, &bk))) return rc;
                if ((rc = c.add_block(F.net, bk, x, out))) return rc;
                x = out;
                continue;
            }
            if ((rc = c.act(t1, x.h, x.w, planes))) return rc;
            if ((rc = c.act(t2, oh, ow, planes))) return rc;
            if ((rc = c.act(out, oh, ow, planes * 4))) return rc;
            if ((rc = c.add_conv(F.net, c1, x, 0, t1, 0))) return rc;
            if ((rc = c.add_conv(F.net, c2, t1, 0, t2, 0))) return rc;
            const Act* idt = &x;
            if (has_ds && c.dual_ok(c3, cd, out)) {
                // relu(bn3(conv3(t2)) + bn(downsample(x))) in one streaming pass: the
                // downsample output never goes through HBM (16-bit and fp32-pair plans)
                if ((rc = c.add_conv_dual(F.net, c3, t2, cd, x, out))) return rc;
                x = out;
                continue;
            }
            if (has_ds) {
                if ((rc = c.act(ds, oh, ow, planes * 4))) return rc;
                if ((rc = c.add_conv(F.net, cd, x, 0, ds, 0))) return rc;
                idt = &ds;
            }
            // relu(bn3(conv3(t2)) + identity)
            if ((rc = c.add_conv(F.net, c3, t2, 0, out, 0, idt, 0, VD_RES_PRE_ACT, 0))) return rc;
            x = out;
        }
        if (li >= 1) feats[li - 1] = x;   // layer2/3/4 -> C3/C4/C5 (config.py:26)
        c.fuse_chains(F.net, layer_begin);   // conv3 -> next conv1 pairs (layer2, chain.hip)
        F.net.stage_end[li + 1] = (int)F.net.ops.size();
    }
    }   // ResNet-50 body

    // ---- FPN ----
    // leaky = 0.1 if out_channels <= 64 else 0 (layers.py:71): LeakyReLU(0.1) for
    // cfg_mnet (64), ReLU for cfg_re50 (256)
    const HT* fo = find_t(W, "fpn.output1.0.weight");
    if (!fo || fo->shape.size() != 4) return vd_set_error(VD_ERR_WEIGHTS, "missing fpn.output1.0.weight");
    const bool fleaky = fo->shape[0] <= 64;
    const int fact = fleaky ? VD_ACT_LEAKY : VD_ACT_RELU;
    const float fslope = fleaky ? 0.1f : 0.f;
    int o1c, o2c, o3c, m1c, m2c;
    if ((rc = c.make_conv_bn(W, "fpn.output1.0.weight", "fpn.output1.1", BN_EPS, 1, 0, fact, fslope, &o1c))) return rc;
    if ((rc = c.make_conv_bn(W, "fpn.output2.0.weight", "fpn.output2.1", BN_EPS, 1, 0, fact, fslope, &o2c))) return rc;
    if ((rc = c.make_conv_bn(W, "fpn.output3.0.weight", "fpn.output3.1", BN_EPS, 1, 0, fact, fslope, &o3c))) return rc;
    if ((rc = c.make_conv_bn(W, "fpn.merge1.0.weight", "fpn.merge1.1", BN_EPS, 1, 1, fact, fslope, &m1c))) return rc;
    if ((rc = c.make_conv_bn(W, "fpn.merge2.0.weight", "fpn.merge2.1", BN_EPS, 1, 1, fact, fslope, &m2c))) return rc;
    const int oc = c.convs[o1c].cout;
    Act o1, o2, o3, m1, m2;
    if ((rc = c.act(o3, feats[2].h, feats[2].w, oc))) return rc;
    if ((rc = c.act(o2, feats[1].h, feats[1].w, oc))) return rc;
    if ((rc = c.act(m2, feats[1].h, feats[1].w, oc))) return rc;
    if ((rc = c.act(o1, feats[0].h, feats[0].w, oc))) return rc;
    if ((rc = c.act(m1, feats[0].h, feats[0].w, oc))) return rc;
    int fpn_at[5];   // op index of o3, o2, m2, o1, m1 (face_lanes)
    fpn_at[0] = (int)F.net.ops.size();
    if ((rc = c.add_conv(F.net, o3c, feats[2], 0, o3, 0))) return rc;
    // output2 = relu(bn(conv(C4))) + nearest_up(output3)   (layers.py:102-103)
    fpn_at[1] = (int)F.net.ops.size();
    if ((rc = c.add_conv(F.net, o2c, feats[1], 0, o2, 0, &o3, 0, VD_RES_POST_ACT, 1))) return rc;
    fpn_at[2] = (int)F.net.ops.size();
    if ((rc = c.add_conv(F.net, m2c, o2, 0, m2, 0))) return rc;
    fpn_at[3] = (int)F.net.ops.size();
    if ((rc = c.add_conv(F.net, o1c, feats[0], 0, o1, 0, &m2, 0, VD_RES_POST_ACT, 1))) return rc;
    fpn_at[4] = (int)F.net.ops.size();
    if ((rc = c.add_conv(F.net, m1c, o1, 0, m1, 0))) return rc;
    if ((int)F.net.ops.size() != fpn_at[4] + 1) return vd_set_error(VD_ERR_STATE, "internal: FPN op count");
    const Act fpn_out[3] = {m1, m2, o3};

    // ---- SSH x3 + fused heads ----
    const bool ssh_fuse = c.tune.ssh_fuse != 0;   // 0: conv3X3 and conv5X5_1 as two convs
    int ssh_b[3], ssh_e[3];                        // op range of each level's SSH + heads
    for (int l = 0; l < 3; ++l) {
        ssh_b[l] = (int)F.net.ops.size();
        const std::string pre = "ssh" + std::to_string(l + 1);
        int s3, s51, s52, s72, s73;
        if ((rc = conv_bn(c, W, pre + ".conv3X3.0.weight", pre + ".conv3X3.1", 1, 1, VD_ACT_RELU, &s3))) return rc;
        // conv5X5_1 / conv7X7_2: LeakyReLU(leaky), leaky = 0.1 if out_channel <= 64 (layers.py:41);
        // the three concat branches take the post-concat ReLU (layers.py:64-65)
        const HT* s3w = find_t(W, pre + ".conv3X3.0.weight");
        const bool sleaky = s3w && s3w->shape.size() == 4 && 2 * s3w->shape[0] <= 64;
        const int sact = sleaky ? VD_ACT_LEAKY : VD_ACT_RELU;
        const float sslope = sleaky ? 0.1f : 0.f;
        if ((rc = c.make_conv_bn(W, pre + ".conv5X5_1.0.weight", pre + ".conv5X5_1.1", BN_EPS, 1, 1, sact, sslope,
                                 &s51)))
            return rc;
        if ((rc = conv_bn(c, W, pre + ".conv5X5_2.0.weight", pre + ".conv5X5_2.1", 1, 1, VD_ACT_RELU, &s52))) return rc;
        if ((rc = c.make_conv_bn(W, pre + ".conv7X7_2.0.weight", pre + ".conv7X7_2.1", BN_EPS, 1, 1, sact, sslope,
                                 &s72)))
            return rc;
        if ((rc = conv_bn(c, W, pre + ".conv7x7_3.0.weight", pre + ".conv7x7_3.1", 1, 1, VD_ACT_RELU, &s73))) return rc;
        const Act& f = fpn_out[l];
        const int c3o = c.convs[s3].cout, c5o = c.convs[s52].cout, c7o = c.convs[s73].cout;
        const int t5c = c.convs[s51].cout;
        Act cat, t5, t7;
        int hoff = 0;   // channel offset of the concat [c3 | c5 | c7] in `cat`
        const int t7c = c.convs[s72].cout;
        if (!sleaky && ssh_fuse && c.tune.ssh_fuse >= 2) {
            // conv5X5_2 and conv7X7_2 both read t5 with ReLU: one conv with Cout c5o + t7c
            // too. cat = [t5 | c3 | c7 | c5 | t7]: the first fused conv writes [t5 | c3],
            // the second [c5 | t7], conv7x7_3 reads t7 and writes c7, and the heads read
            // [c3 | c7 | c5] with their input channels permuted to that order.
            int s351, s5272;
            if ((rc = c.make_conv_bn_cat(W, {{pre + ".conv5X5_1.0.weight", pre + ".conv5X5_1.1"},
                                             {pre + ".conv3X3.0.weight", pre + ".conv3X3.1"}},
                                         BN_EPS, 1, 1, VD_ACT_RELU, 0.f, &s351)))
                return rc;
            if ((rc = c.make_conv_bn_cat(W, {{pre + ".conv5X5_2.0.weight", pre + ".conv5X5_2.1"},
                                             {pre + ".conv7X7_2.0.weight", pre + ".conv7X7_2.1"}},
                                         BN_EPS, 1, 1, VD_ACT_RELU, 0.f, &s5272)))
                return rc;
            if ((rc = c.act(cat, f.h, f.w, t5c + c3o + c7o + c5o + t7c))) return rc;
            const int o_c7 = t5c + c3o, o_c5 = o_c7 + c7o, o_t7 = o_c5 + c5o;
            if ((rc = c.add_conv(F.net, s351, f, 0, cat, 0))) return rc;
            if ((rc = c.add_conv(F.net, s5272, cat, 0, cat, o_c5))) return rc;
            if ((rc = c.add_conv(F.net, s73, cat, o_t7, cat, o_c7))) return rc;
            std::vector<int> perm(c3o + c5o + c7o);   // packed [c3 | c7 | c5] <- tensors' [c3 | c5 | c7]
            for (int i = 0; i < c3o; ++i) perm[i] = i;
            for (int i = 0; i < c7o; ++i) perm[c3o + i] = c3o + c5o + i;
            for (int i = 0; i < c5o; ++i) perm[c3o + c7o + i] = c3o + i;
            int hc;
            const std::string L = std::to_string(l);
            if ((rc = c.make_conv_cat(W,
                                      {"BboxHead." + L + ".conv1x1.weight", "ClassHead." + L + ".conv1x1.weight",
                                       "LandmarkHead." + L + ".conv1x1.weight"},
                                      {"BboxHead." + L + ".conv1x1.bias", "ClassHead." + L + ".conv1x1.bias",
                                       "LandmarkHead." + L + ".conv1x1.bias"},
                                      VD_ACT_NONE, &hc, &perm)))
                return rc;
            if (c.convs[hc].cout != 32) return vd_set_error(VD_ERR_WEIGHTS, "heads of level %d: %d channels != 32", l, c.convs[hc].cout);
            if ((rc = c.act(F.heads[l], f.h, f.w, 32, true))) return rc;
            if ((rc = c.add_conv(F.net, hc, cat, t5c, F.heads[l], 0))) return rc;
            ssh_e[l] = (int)F.net.ops.size();
            continue;
        }
        if ((rc = c.act(t7, f.h, f.w, t7c))) return rc;
        if (!sleaky && ssh_fuse) {
            // conv5X5_1 and conv3X3 read the same input with the same activation
            // (ReLU: conv3X3's own, after the concat): one conv with Cout t5c + c3o
            // writing [t5 | c3] into cat = [t5 | c3 | c5 | c7], so the input is read once
            int s351;
            if ((rc = c.make_conv_bn_cat(W, {{pre + ".conv5X5_1.0.weight", pre + ".conv5X5_1.1"},
                                             {pre + ".conv3X3.0.weight", pre + ".conv3X3.1"}},
                                         BN_EPS, 1, 1, VD_ACT_RELU, 0.f, &s351)))
                return rc;
            if ((rc = c.act(cat, f.h, f.w, t5c + c3o + c5o + c7o))) return rc;
            t5 = cat;
            hoff = t5c;
            if ((rc = c.add_conv(F.net, s351, f, 0, cat, 0))) return rc;
        } else {
            if ((rc = c.act(cat, f.h, f.w, c3o + c5o + c7o))) return rc;
            if ((rc = c.act(t5, f.h, f.w, t5c))) return rc;
            if ((rc = c.add_conv(F.net, s3, f, 0, cat, 0))) return rc;
            if ((rc = c.add_conv(F.net, s51, f, 0, t5, 0))) return rc;
        }
        if ((rc = c.add_conv(F.net, s52, t5, 0, cat, hoff + c3o))) return rc;
        if ((rc = c.add_conv(F.net, s72, t5, 0, t7, 0))) return rc;
        if ((rc = c.add_conv(F.net, s73, t7, 0, cat, hoff + c3o + c5o))) return rc;
        int hc;
        const std::string L = std::to_string(l);
        if ((rc = c.make_conv_cat(W,
                                  {"BboxHead." + L + ".conv1x1.weight", "ClassHead." + L + ".conv1x1.weight",
                                   "LandmarkHead." + L + ".conv1x1.weight"},
                                  {"BboxHead." + L + ".conv1x1.bias", "ClassHead." + L + ".conv1x1.bias",
                                   "LandmarkHead." + L + ".conv1x1.bias"},
                                  VD_ACT_NONE, &hc)))
            return rc;
        if (c.convs[hc].cout != 32) return vd_set_error(VD_ERR_WEIGHTS, "heads of level %d: %d channels != 32", l, c.convs[hc].cout);
        if ((rc = c.act(F.heads[l], f.h, f.w, 32, true))) return rc;
        if ((rc = c.add_conv(F.net, hc, cat, hoff, F.heads[l], 0))) return rc;
        ssh_e[l] = (int)F.net.ops.size();
    }
    if (c.tune.ssh_side && (rc = c.face_lanes(fpn_at, ssh_b, ssh_e))) return rc;

    // ---- anchors (anchors.py:22-41, Python doubles -> float32) ----
    static const int steps[3] = {8, 16, 32};
    static const int min_sizes[3][2] = {{16, 32}, {64, 128}, {256, 512}};
    std::vector<float> anc;
    int A = 0;
    for (int l = 0; l < 3; ++l) {
        const int fh = (H + steps[l] - 1) / steps[l], fw = (Wd + steps[l] - 1) / steps[l];
        if (fh != F.heads[l].h || fw != F.heads[l].w)
            return vd_set_error(VD_ERR_ARG, "anchor grid %dx%d != head %dx%d", fh, fw, F.heads[l].h, F.heads[l].w);
        F.loff[l] = A;
        for (int i = 0; i < fh; ++i)
            for (int j = 0; j < fw; ++j)
                for (int k = 0; k < 2; ++k) {
                    const double ms = min_sizes[l][k];
                    anc.push_back((float)((j + 0.5) * steps[l] / Wd));
                    anc.push_back((float)((i + 0.5) * steps[l] / H));
                    anc.push_back((float)(ms / Wd));
                    anc.push_back((float)(ms / H));
                    ++A;
                }
    }
    F.A = A;
    if ((rc = c.dalloc((void**)&F.anchors, anc.size() * 4))) return rc;
    VD_CHECK_HIP(hipMemcpy(F.anchors, anc.data(), anc.size() * 4, hipMemcpyHostToDevice));
    if ((rc = vd_alloc_post(c, F.post, A, A))) return rc;   // a frame keeps at most A faces
    F.net.amax = c.amax_region(0);
    F.net.amax_bytes = F.net.amax ? c.amax_region_bytes() : 0;
    F.loaded = true;
    return VD_OK;
}

int vd_alloc_post(Ctx& c, PostScratch& ps, int A, int kcap) {
    const size_t B = c.cfg.max_batch;
    int P = 1;
    while (P < A) P <<= 1;
    ps.sort_cap = P;
    int rc;
    if ((rc = c.dalloc((void**)&ps.keys, B * A * 8))) return rc;
    if ((rc = c.dalloc((void**)&ps.count, B * 4))) return rc;
    if ((rc = c.dalloc((void**)&ps.box, B * A * 16))) return rc;
    if ((rc = c.dalloc((void**)&ps.cls, B * A * 4))) return rc;
    if ((rc = c.dalloc((void**)&ps.nbox, B * A * 16))) return rc;
    if ((rc = c.dalloc((void**)&ps.area, B * A * 4))) return rc;
    if ((rc = c.dalloc((void**)&ps.sort, B * (size_t)P * 8))) return rc;
    if ((rc = c.dalloc((void**)&ps.supp, B * A))) return rc;
    ps.kcap = kcap;
    if ((rc = c.dalloc((void**)&ps.kcount, B * 4))) return rc;
    if ((rc = c.dalloc((void**)&ps.kxyxy, B * kcap * 16))) return rc;
    if ((rc = c.dalloc((void**)&ps.kxyxy_f, B * kcap * 16))) return rc;
    if ((rc = c.dalloc((void**)&ps.kscore, B * kcap * 4))) return rc;
    if ((rc = c.dalloc((void**)&ps.klabel, B * kcap * 4))) return rc;
    VD_CHECK_HIP(hipMemset(ps.kcount, 0, B * 4));
    return VD_OK;
}

void vd_post_keep_args(PostScratch& ps, PostArgs& p, int n) {
    p.kcap = ps.kcap;
    p.k_count = ps.kcount; p.k_xyxy = ps.kxyxy; p.k_xyxy_f = ps.kxyxy_f; p.k_score = ps.kscore; p.k_label = ps.klabel;
    ps.kn = n;
}
