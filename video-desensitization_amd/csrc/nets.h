// nets.h — host-side context, network plans and builders (internal).
#pragma once
#include "../../include/vdmi.h"
#include "vd_common.h"

#include <mutex>
#include <string>
#include <unordered_map>
#include <utility>
#include <map>
#include <vector>

struct HT {   // host tensor from the VDW1 container
    std::vector<int> shape;
    std::vector<float> data;
};
using WMap = std::unordered_map<std::string, HT>;
int vd_parse_vdw1(const void* blob, size_t bytes, WMap& out);
const HT* find_t(const WMap& W, const std::string& k);
void vd_resize_mode(int ih, int iw, int nh, int nw, int* mode, double* sx, double* sy);

struct Act {          // NHWC activation buffer sized for cfg.max_batch frames
    void* p = nullptr;
    int h = 0, w = 0, c = 0;   // c = channel stride
    bool f32 = false;
    // fp16-pair plan (f32_split = 2): per-frame running max |x| [max_batch] that every
    // producer folds its outputs into (conv_x6.hip AmaxTrack), or a static bound
    // for the letterboxed canvas (amax NULL)
    unsigned* amax = nullptr;
    float bound = 0.f;
    bool exact16 = false;      // every value an integer of |x| <= 2048 (the face letterbox canvas)
};

struct Conv {
    int cin = 0, cin_pad = 0, cout = 0, npad = 0, kh = 0, kw = 0, stride = 1, pad = 0, kpad = 0, act = 0;
    float slope = 0.f;
    void* w = nullptr;
    void* wx3 = nullptr;       // fp32 + f32_split: [npad][kpad/32][3][32] bf16 / [..][2][32] fp16 planes (conv_x6.hip)
    float* scale_x = nullptr;  // fp16 pairs: BN scale times the row's 2^-e
    void* wx3_chain = nullptr; // fp16 pairs as chain32.hip's conv1': K permuted inside each 32-step
    int split = 0;             // fp32: VdTune::f32_split when the weights were packed
    float* scale = nullptr;
    float* shift = nullptr;
    double flops_per_px = 0;   // algorithmic FLOPs per output pixel (real Cin, no padding)
    int grp_co = 0, grp_ci = 0; // grouped (conv_x6_halo only): rows [g grp_co, +grp_co) read input channels g grp_ci + [0, cin)
};

// One fused layer1 bottleneck (block.hip, block.cpp): the per-conv bf16 weights
// of conv1/conv2/conv3(/downsample) repacked for the fused kernel.
struct Block {
    int cin = 0, ds = 0;
    bool f32 = false;                         // fp32 plan (block32.hip): fp16-pair planes / fragments
    int c1 = -1, c2 = -1, c3 = -1, cd = -1;   // the per-conv plans (flops, unfused fallback)
    void* w1 = nullptr;
    void* w2 = nullptr;
    void* w3 = nullptr;
    void* wd = nullptr;
    float* bn = nullptr;
};

// Depthwise 3x3 conv + BN + activation (dwconv.hip): MobileNetV1 conv_dw.
struct DwConv {
    int c = 0, stride = 1, act = 0;
    float slope = 0.f;
    void* w = nullptr;                 // [9][c] in the compute type
    float* scale = nullptr;
    float* shift = nullptr;
};

enum { OP_CONV = 0, OP_MAXPOOL = 1, OP_UPSAMPLE = 2, OP_BLOCK = 3, OP_STEMPOOL = 4, OP_DWCONV = 5, OP_CHAIN = 6 };

struct Op {
    int kind = OP_CONV;
    int conv = -1;
    Act x; int xcoff = 0;
    Act y; int ycoff = 0;
    Act r; int rcoff = 0; int rmode = 0; int rup = 0;
    int conv2 = -1; Act x2;            // fused second 1x1 conv (downsample branch), summed pre-activation
    int ch = 0, k = 0, s = 0, p = 0;   // maxpool / upsample
    int blk = -1;                      // OP_BLOCK: index into Ctx::blocks (x -> y)
    void* wf = nullptr;                // OP_STEMPOOL: conv's weight fragments (conv = the stem conv)
    Act y2;                            // OP_CHAIN: conv = conv3 (x -> y, identity r), conv2 = next conv1 (y -> y2)
    int lane = 0;                      // 1: runs on Ctx::stream_side (face SSH levels 1-2)
    int dep = -1;                      // op index (other lane) whose completion this op waits for
};

struct Net {
    std::vector<Op> ops;
    unsigned* amax = nullptr;                        // fp16-pair plan: this net's max slots, zeroed per run
    size_t amax_bytes = 0;
    int stage_end[8] = {0, 0, 0, 0, 0, 0, 0, 0};   // op index after each backbone stage (face: 0=stem,1..4=layerN)
    int conv_fam = 0;                                // timing family of its convs (0 face, 5 plate)
};

struct PostScratch {   // per-net candidate / NMS scratch sized for max_batch x A
    uint64_t* keys = nullptr;
    int* count = nullptr;
    float4* box = nullptr;
    int* cls = nullptr;
    float4* nbox = nullptr;
    float* area = nullptr;
    uint64_t* sort = nullptr;
    uint8_t* supp = nullptr;
    int sort_cap = 0;
    // the last call's complete keep lists [max_batch][kcap] (library-owned): the
    // mosaic reads these, never the caller's cap-limited copies; vd_read_boxes
    // hands them out
    int kcap = 0;
    int* kcount = nullptr;
    int* kxyxy = nullptr;
    float* kxyxy_f = nullptr;
    float* kscore = nullptr;
    int* klabel = nullptr;
    int kn = 0;                        // frames in the last call
};

struct FaceNet {
    bool loaded = false;
    int in_h = 640, in_w = 640;
    bool s2d = false;               // 16-bit / fp32-pair plans: stem input in space-to-depth form (pre.hip letterbox_s2d_kernel)
    bool mnet = false;              // MobileNetV1-0.25 backbone (cfg_mnet) instead of ResNet-50
    Act input;
    Net net;
    Act heads[3];
    int loff[3] = {0, 0, 0};
    int A = 0;
    float* anchors = nullptr;
    PostScratch post;
};

struct PlateNet {
    bool loaded = false;
    int nc = 1;
    int imgsz = 640;
    int hstride = 0;                // head channel stride (64 DFL + nc, padded to 8)
    Act input;                      // letterboxed canvas, allocated for imgsz x imgsz
    bool s2d = false;               // 16-bit / fp32-pair plans: canvas in space-to-depth form, model.0 as a 2x2 conv
    std::vector<std::pair<std::string, Act>> bufs;   // named activation buffers (max canvas)
    std::vector<std::pair<std::string, int>> conv_idx;
    std::vector<std::pair<long long, Net>> plans;    // per canvas (h<<32|w)
    Act head[3];
    int A_max = 0;
    PostScratch post;
    // current call
    int ch = 0, cw = 0, A = 0, lh[3] = {0, 0, 0}, lw[3] = {0, 0, 0}, loff[3] = {0, 0, 0};
};

struct BoxTargets {
    int cap = 0;
    int* count = nullptr;
    int* xyxy = nullptr;
    float* xyxy_f = nullptr;
    float* score = nullptr;
    int* label = nullptr;
};

struct TimedEv {
    hipEvent_t a, b;
    int fam;
    double work;
};

struct Ctx {
    vd_cfg cfg{};
    int device = 0;
    bool f32 = false;
    bool f16 = false;                             // VD_PREC_FP16: fp16 operands/activations (the bf16 plan's kernels)
    VdTune tune;                                  // kernel-selection switches (vd_set_option)
    hipStream_t stream = nullptr, own_stream = nullptr;
    hipStream_t stream2 = nullptr;               // plate branch runs beside the face branch
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    hipStream_t stream_side = nullptr;           // the face net's second lane (SSH levels 1-2 beside level 0)
    std::vector<hipEvent_t> lane_ev;             // per face op: completion event for the other lane
    hipEvent_t ev_side = nullptr;                // side lane done (joined before the face decode)
    hipEvent_t ev_half = nullptr;                // option face_groups: fork of the frame groups
    std::vector<hipStream_t> group_streams;      // option face_groups: streams of frame groups 1..G-1
    std::vector<hipEvent_t> group_events;        //   and their completion events (joined by the context stream)
    std::map<int, unsigned*> amax_snaps;         // per conv: its input's range slots frozen (in-place concat)
    int fork_at = -1;                                // run_ops records ev_fork after this many face ops
    std::mutex mu;
    std::vector<void*> allocs;
    std::vector<Conv> convs;
    std::vector<Block> blocks;
    std::vector<DwConv> dwconvs;
    FaceNet face;
    PlateNet plate;
    void* stage_in = nullptr;  size_t stage_in_bytes = 0;
    void* stage_out = nullptr; size_t stage_out_bytes = 0;
    void* stage_box = nullptr; size_t stage_box_bytes = 0;
    void* stage_box2 = nullptr; size_t stage_box2_bytes = 0;
    void* mosaic_table = nullptr; size_t mosaic_table_bytes = 0;
    // JPEG frame decode (jpeg_host.cpp): pinned host staging, device copy, planes
    void* jpeg_host = nullptr; size_t jpeg_host_bytes = 0;
    void* jpeg_dev = nullptr; size_t jpeg_dev_bytes = 0;
    void* jpeg_planes = nullptr; size_t jpeg_planes_bytes = 0;
    hipEvent_t jpeg_ev = nullptr;                 // last H2D out of jpeg_host / jenc_host
    // device entropy decode (jpeg_dec.hip): pinned segments + tables + metadata, device copy, dense blocks
    void* jdec_host = nullptr; size_t jdec_host_bytes = 0;
    void* jdec_dev = nullptr; size_t jdec_dev_bytes = 0;
    void* jdec_work = nullptr; size_t jdec_work_bytes = 0;
    int jdec_passes = 0;                          // sync passes of the last device decode (test hook)
    // JPEG frame encode (jpeg_enc.cpp): device coefficients + tables, pinned host copy
    void* jenc_dev = nullptr; size_t jenc_dev_bytes = 0;
    void* jhuf_dev = nullptr; size_t jhuf_dev_bytes = 0;   // device entropy stage buffers
    void* jseg_host = nullptr; size_t jseg_host_bytes = 0; // pinned: packed entropy-coded segments
    void* jenc_host = nullptr; size_t jenc_host_bytes = 0;
    int jpeg_threads = 16;                        // host entropy-decode threads
    // fp16-pair plan: per-frame activation max slots, one region per network (face 0,
    // plates 1) of kAmaxActs activations x max_batch frames
    static constexpr int kAmaxActs = 256;
    unsigned* amax_pool = nullptr;
    int amax_owner = 0;
    int amax_next[2] = {0, 0};
    int amax_begin(int owner);                    // builders: slots of `owner` restart
    unsigned* amax_region(int owner) const { return amax_pool ? amax_pool + (size_t)owner * kAmaxActs * cfg.max_batch : nullptr; }
    size_t amax_region_bytes() const { return (size_t)kAmaxActs * cfg.max_batch * 4; }
    bool timing = false;
    std::vector<TimedEv> ev_pool;
    size_t ev_used = 0;

    int dalloc(void** p, size_t bytes);
    int act(Act& a, int h, int w, int c, bool f32out = false, bool half = false);   // half: 2-byte elements
    int ensure_staging(void** p, size_t* have, size_t need);
    int ensure_pinned(void** p, size_t* have, size_t need);
    int upload_conv(Conv& cv, const std::vector<float>& w_oihw, const std::vector<float>& scale,
                    const std::vector<float>& shift);
    int make_conv_bn(const WMap& W, const std::string& wkey, const std::string& bn, float eps, int stride, int pad,
                     int act, float slope, int* out_idx);
    // convs + BatchNorms {(wkey, bn)} concatenated along Cout (same input, kernel, stride, pad)
    int make_conv_bn_cat(const WMap& W, const std::vector<std::pair<std::string, std::string>>& parts, float eps,
                         int stride, int pad, int act, float slope, int* out_idx);
    int make_conv_cat(const WMap& W, const std::vector<std::string>& wkeys, const std::vector<std::string>& bkeys,
                      int act, int* out_idx,
                      const std::vector<int>* cin_perm = nullptr);
    int add_conv_dual(Net& net, int ci, const Act& x, int c2, const Act& x2, Act& y);
    bool dual_ok(int ci, int c2, const Act& y) const;
    int add_conv(Net& net, int ci, const Act& x, int xcoff, Act& y, int ycoff, const Act* res = nullptr,
                 int rcoff = 0, int rmode = 0, int rup = 0);
    bool block_ok(int c1, int c2, int c3, int cd, const Act& x) const;
    int make_block(int c1, int c2, int c3, int cd, int* idx);
    int add_block(Net& net, int bi, const Act& x, Act& y);
    int run_block_op(const Op& op, int f0, int n, int fam = 0);
    int add_stem_pool(Net& net, int ci, const Act& x, Act& y);
    int make_dwconv_bn(const WMap& W, const std::string& wkey, const std::string& bn, float eps, int stride, int act,
                       float slope, int* idx);
    int add_dwconv(Net& net, int di, const Act& x, Act& y);
    int run_dwconv_op(const Op& op, int f0, int n);
    int run_chain_op(const Op& op, int f0, int n, int fam = 0);
    void fuse_chains(Net& net, size_t begin);
    int run_stem_pool_op(const Op& op, int f0, int n, int fam = 0);
    void t_begin(int fam, double work);
    void t_end();
    int run_conv_op(const Op& op, int f0, int n, int fam = 0);
    int run_ops(const Net& net, int b, int e, int f0, int n);
    int face_lanes(const int (&fpn)[5], const int (&ssh_b)[3], const int (&ssh_e)[3]);
    int chain32_weights(Conv& c1);
    void fuse_chains32(Net& net, size_t begin);
    int run_net(const Net& net, int n, int mb = 0, int split = 0);
    const uint8_t* frames_to_device(const uint8_t* frames, int n, int h, size_t pitch, int where, int* rc);
    int check_frames(int n, int h, int w, size_t pitch);
    int box_targets(vd_boxes* out, int n, BoxTargets& t);
    int box_finish(vd_boxes* out, int n, const BoxTargets& t);
    int host_box_staging(void** buf, size_t* have, int cap, int n, BoxTargets& t);
    int face_letterbox(const uint8_t* dframes, int n, int h, int w, size_t pitch);
    void face_letterbox_args(const uint8_t* dframes, int n, int h, int w, size_t pitch, LetterboxArgs* a);
    int face_forward(int n);
    int face_post(int n, int img_h, int img_w, const BoxTargets& t);
    int launch_mosaic(const uint8_t* in, uint8_t* out, int n, int h, int w, size_t pitch, const int* cnt0,
                      const int* xy0, int cap0, const int* cnt1, const int* xy1, int cap1, int level);
};

int vd_alloc_post(Ctx& ctx, PostScratch& ps, int A, int kcap);
void vd_post_keep_args(PostScratch& ps, PostArgs& p, int n);
int vd_build_face(Ctx& ctx, const WMap& W);
int vd_build_plate(Ctx& ctx, const WMap& W);
// letterboxed: the canvas was already written (vd_launch_letterbox_pair in vd_process)
int vd_plate_forward(Ctx& ctx, const uint8_t* dframes, int n, int h, int w, size_t pitch, bool letterboxed = false);
int vd_plate_letterbox_args(Ctx& ctx, const uint8_t* dframes, int n, int h, int w, size_t pitch, LetterboxArgs* a);
int vd_plate_post(Ctx& ctx, int n, int img_h, int img_w, const BoxTargets& t);
