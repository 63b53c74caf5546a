// vd_common.h — internal types shared by the HIP kernels and the runtime.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>
#include <stddef.h>

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));

typedef unsigned vd_u32x4 __attribute__((ext_vector_type(4)));

// The 16-bit operand type of the bf16 plan (F16 = false) and the fp16 plan (VD_PREC_FP16,
// F16 = true): element type, 8-vector, the 16x16x32 matrix-core product, and the two
// elements of a packed 32-bit word as f32. Conversions to T are round-to-nearest-even.
template <bool F16> struct Half16;
template <> struct Half16<false> {
    typedef __bf16 T;
    typedef bf16x8_t V8;
    static __device__ __forceinline__ f32x4_t mfma(const vd_u32x4& a, const vd_u32x4& b, const f32x4_t& c) {
        return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b),
                                                       c, 0, 0, 0);
    }
    static __device__ __forceinline__ float lo(unsigned u) { return __uint_as_float(u << 16); }
    static __device__ __forceinline__ float hi(unsigned u) { return __uint_as_float(u & 0xFFFF0000u); }
};
template <> struct Half16<true> {
    typedef _Float16 T;
    typedef f16x8_t V8;
    static __device__ __forceinline__ f32x4_t mfma(const vd_u32x4& a, const vd_u32x4& b, const f32x4_t& c) {
        return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8_t, a), __builtin_bit_cast(f16x8_t, b),
                                                      c, 0, 0, 0);
    }
    static __device__ __forceinline__ float lo(unsigned u) {
        return (float)__builtin_bit_cast(_Float16, (unsigned short)(u & 0xFFFFu));
    }
    static __device__ __forceinline__ float hi(unsigned u) { return (float)__builtin_bit_cast(_Float16, (unsigned short)(u >> 16)); }
};

enum VdAct { VD_ACT_NONE = 0, VD_ACT_RELU = 1, VD_ACT_LEAKY = 2, VD_ACT_SILU = 3 };
enum VdResMode { VD_RES_NONE = 0, VD_RES_PRE_ACT = 1, VD_RES_POST_ACT = 2 };

// Kernel-selection switches of one context. The defaults ARE the production plan;
// vd_set_option (include/vdmi.h) changes them per context for A/B measurements and
// for tests that force a kernel form onto small shapes. Plan-time switches
// (block_fuse, chain, stem_pool, ssh_fuse, plate_s2d) take effect at the next
// vd_load_weights; the others at the next launch. Nothing is read from the
// environment.
struct VdTune {
    int conv_stream = 1;      // streaming 1x1 kernel (conv1x1.hip) for K in {64,128,256}
    int conv_stream512 = 1;   //   ... and K = 512
    int conv_dual = 1;        // conv3 + downsample as one streaming launch
    int conv_taps = 1;        // streaming taps kernel for small K (YOLO)
    int conv_n192 = 1;        // 192-wide N tile for Cout 129..192 (fused SSH conv)
    int conv_small = 512;     // below this many 128-row tiles the GEMM takes 64-row tiles
    int conv_big = 100;       // min 256x256 tiles for the phased kernel (0: off)
    int conv_big_kmin = 512;  // min K for the phased kernel
    int stream_ntt = 16;      // streaming 1x1: 256-channel slices where Cout allows (8: 128)
    int lb_pair = 1;          // one letterbox launch for both canvases when geometry allows
    int mosaic_map = 1;       // mosaic output pass: per-band vector maps (0: generic path)
    int mosaic_nt = 0;        //   non-temporal output stores (1), and source loads (3)
    int mosaic_cells = 32;    //   cell-table kernel: workgroups per frame
    int mosaic_gather = 0;    //   fused output pass: a thread's band cells walked, then their loads issued together
    int mosaic_rows = 0;      //   fused output pass: rows per band (4 / 8 / 16 / 24 / 32; 0 = auto: 4 for rows
                              //   of >= 8 KB (4K), else 8)
    int mosaic_fused = 1;     //   one launch: the output pass computes its bands' cell colours itself (0: cell kernel + output pass)
    int block_fuse = 1;       // plan: fused layer1 bottlenecks (block.hip)
    int block32_xd = 2;       //   block32 stage-1 x loads in flight + 1 (register sets: 2, 3, 4)
    int block32_dbg = 0;      //   timing-only (vdt_set_debug, never vd_set_option): skip block32 stages (bits: 1 S1, 2 S2, 4 S3 math, 8 S3 stores, 16 S3 identity)
    int block32_pipe = 1;     //   block32 (CIN 256): producer / consumer wave groups on consecutive tiles (0: one group)
    int block_fuse32 = 1;     // plan, fp32 (fp16 pairs): fused layer1 bottlenecks (block32.hip)
    int chain = 2;            // plan: conv3 + next conv1 as one kernel (chain.hip; fp32: chain32.hip: 2 = layer2,
                              //   1 = layer2 + layer3 -- level on the grouped headline, slower per launch)
    int stem_pool = 1;        // plan: stem conv + maxpool (stem.hip)
    int ssh_fuse = 2;         // plan: SSH conv3X3 + conv5X5_1 as one conv (2: and conv5X5_2 + conv7X7_2)
    int plate_s2d = 1;        // plan: YOLO space-to-depth stem input
    int jenc_gpu = 1;         // vd_jpeg_encode: Huffman coding on the device (0: host threads)
    int jdec_gpu = 1;         // vd_jpeg_decode: entropy decode on the device (0: host threads)
    int jdec_sync = 128;      //   states recorded per chunk: passes stop at the previous trajectory (0: off)
    int jdec_chunk = 1024;    //   raw scan bytes per decoding thread (tests force small chunks)
    int jdec_group = 4;       //   resynchronisation passes launched between host convergence checks
    int ssh_side = 0;         // 1: face SSH levels 1-2 (+ heads) on a second stream beside FPN merge / level 0
                              //   (at weight load; measured -0.1 ms/step, but overlapping launches inflate
                              //   the per-launch durations behind `roofline`: off by default)
    int chain_gpw = 1;        // chain32.hip layer2: 16-pixel groups per wave (2: 256-pixel super-groups)
    int det_group = 1;        // plan (fp32): the Detect heads' cv2.i.1 + cv3.i.1 as one grouped 3x3 conv
    int plate_s2d32 = 1;      // fp32 plan: the plate stem on the fp16 space-to-depth canvas (with plate_s2d)
    int face_groups = 2;      // face net as G frame groups on G streams (the tails of one group's launches
                              //   fill with the others'; bit-identical; 0 / 1: one launch over the batch)
    int plate_detect_early = 1; // plan: each YOLO Detect level right after its P level (0: all three at the end)
    int mosaic_early = 1;     // vd_process without MOSAIC_PLATES: the face mosaic runs before the plate branch joins
    int plate_stage = 3;      // plate branch starts after face stage N (0: with the stem; 1-4: after
                              //   layerN; 5: after the whole face net). After layer3 its HBM-bound
                              //   convs overlap the MFMA-bound late face layers: 30.8 -> 30.0 ms/step
    int x6_stream = 1;        // fp32 split: streaming 1x1 kernel for K in {64, 128, 256}
    int x6_stream_rl = 1;     //   streaming 1x1 with a residual: one input register set refilled per k-step, the
                              //   residual loaded at the top of each pixel group (beside the MFMAs), not in the epilogue
                              //   (2: also the layers without a residual -- measured level, r06ag)
    int x6_stream_silu = 1;   //   fp16 pairs: also SiLU 1x1 convs (YOLO C2f / SPPF) with K in {32..256}
    int x6_stream256 = 2;     //   fp16 pairs, Cout % 256 == 0: 256-channel slices for K = 64 (2: and K = 128;
                              //   each pixel read by half as many workgroups: faces 27.31 -> 26.96 ms/step)
    int x6_small_k = 256;     // fp32 split: K at or below which the small single-stage tile runs
    int x6_small_tiles = 512; //   ... and big-tile grids smaller than this (0 / 0: big tile always)
    int x6_small_k2 = 1 << 20;//   fp16 pairs: K at or below which N <= 64 layers take the small tile
    int x6_bn256 = 1;         // fp16 pairs: 256 x 256 tile for Cout % 256 == 0
    int x6_exact = 1;         // fp16 pairs: one A plane for inputs exact in fp16 (the face stem)
    int x6_mid = 512;         // fp16 pairs: 1x1 Cout-128 convs with K <= this on the 128 x 128 two-stage tile (0: off)
    int x6_mf32 = 0;          // fp16 pairs: 256 x {256,128} tiles on v_mfma_f32_32x32x16_f16 (else 16x16x32)
    int x6_tail = 0;          // fp16 pairs, big tiles: rows past the last full round of 256-row tiles on
                              //   narrower tiles (1: BN/2, 2: BN/4 columns, 0: off); N splits keep every
                              //   output's K order, so results do not depend on the split. Measured
                              //   slower (27.6 -> 28.5 / 28.9 ms per step for 1 / 2): the narrow tiles
                              //   fetch more per FLOP, and a partial round's workgroups run faster alone
    int x6_halo = 2;          // fp16 pairs, 3x3 stride-1 convs: input split once per 32-channel chunk
                              //   over the tile's linear halo (conv_x6_halo_kernel); 2: three B stages, 1: two
    int x6_halo_narrow = 1;   // ... also for Cout <= 64 (N tiles of 32 / 64)
    int x6_halo_s2 = 1;       // ... also 3x3 stride-2 convs (phase halos; Cout > 32)
    int x6_adepth = 2;        // A register sets of the 256 x {128, 64, 32} fp16-pair tiles (2 or 4; 4 measured level)
    int x6_slots = 0;         //   workgroup slots of one round (0: the CU count; tests force small values)
    int x6_halo_1b = 1;       // halo tiles with two B stages (wide frames): one barrier per step (0: two)
    int x6_gemm_uni = 2;      // 1x1 GEMM two-stage loop: the same loads / DMAs every K tile (past the end: the
                              //   last tile again), so the compiler's register waits stay off the next tile
                              //   (0: round-5 loop; 2: also one barrier per K tile)
    int x6_gemm_pf = 1;       // GEMM tiles with wide wave tiles (TN > TM): the same pipelined B-fragment reads
    int x6_halo_n64 = 0;      //   halo tiles: Cout-128 3x3 layers with K <= this as two 64-wide N tiles (0: off)
    int x6_halo_pf = 1;       //   halo tiles (128-256 wide): B fragments of block j + 1 read before block j's MFMAs
    int x6_halo_dma = 2;      //   halo tiles: where a K step issues the B DMA two steps ahead (0 after the
                              //   barrier, 1 after the step's MFMAs, 2 one piece between MFMA groups)
    int x6_tr_epi = 1;        // TR register epilogue: 1 = residual / BN rows of column pair jp + 1 loaded before pair
                              //   jp's stores (buffer ops, straight-line), 0 = the round-5 row-by-row form
    int x6_halo_tr = 2;       // fp32 plan: halo 3x3 tiles with D^T accumulators and the register epilogue
                              //   (1: the 128-256-wide tiles, 2: all; bit-identical)
    int x6_one = 1;           // fp16 pairs, GEMM tiles: 1x1 convs load A at row offset + scalar K offset (no tap stepping)
    int x6_taps = 1;          // fp32 plan: narrow KxK YOLO layers (K <= 288) on the streaming TAPS form
    int x6_gemm1x1 = 1;       // fp16 pairs: GEMM 1x1 convs on the TR tiles (D^T accumulators, register epilogue;
                              //   2: also the streaming form's K <= 256 layers, 0: off)
    int x6_dbg = 0;           // experiments (vdt_set_debug / tools/x6bench): 1 = no epilogue (WRONG results), 2 = runtime vmcnt waits
    int f32_split = 2;        // plan (fp32, at weight load): 2 = operands scaled by powers of two
                              //   and split into fp16 pairs, 3 products on the f16 matrix cores;
                              //   1 = exact 3-term bf16 split, 6 products (conv_x6.hip);
                              //   0 = exact-f32 v_mfma_f32_16x16x4_f32 (conv.hip)
};

// Implicit-GEMM convolution parameters (device side). Activations are NHWC with
// an explicit channel stride (ld) and channel offset (coff) so a conv can read
// a channel slice of a concat buffer and write into one (SSH concat,
// layers.py:64; YOLO C2f/Concat).
struct ConvArgs {
    const void* x;  int xh, xw, ldx, xcoff;     // input  [B][xh][xw][ldx]
    const void* w;                               // packed weights [Npad][Kpad]
    const float* scale; const float* shift;      // BN eval as y = acc*scale + shift (len Npad)
    const void* res; int res_ld, res_coff, res_up;  // residual NHWC; res_up: 1 = nearest 2x source
    int rh, rw;                                  // residual spatial dims
    void* y;  int yh, yw, ldy, ycoff;            // output [B][yh][yw][ldy]
    int B, cin_pad, cout, kpad;                  // cin_pad: channels per tap in the K order
    int kh, kw, stride, pad;
    int M;                                       // B*yh*yw
    int act; float slope; int res_mode; int out_f32;
    int f16;                                     // 16-bit type is fp16 (VD_PREC_FP16), else bf16
    int ntiles_n;                                // ceil(cout / BN)
    // optional second 1x1 conv summed before the activation (bottleneck conv3 +
    // downsample in one pass): y = act(acc*scale + shift + acc2*scale2 + shift2)
    const void* x2; int xh2, xw2, ldx2, xcoff2, stride2;
    const void* w2; const float* scale2; const float* shift2; int cin2_pad, kpad2;
    const VdTune* tune;                          // host-side kernel selection (never read on the device)
    const void* wx3;                             // fp32: split weights (conv_x6.hip: 3 bf16 / 2 fp16 planes), or NULL
    // f32_split = 2 (fp16 pair): per-channel BN scale with the weight rows' 2^-e folded in,
    // the input's running max |x| (device slot, or a static bound when NULL) and the
    // output's slot (atomic max of |y|; NULL: not tracked)
    const float* scale_x;
    int f32_split;                               // the conv's weight format (Conv::split at load)
    const unsigned* xmax; float xbound;
    unsigned* ymax;
    // fp16 pairs, fused downsample (x2): its split weights, rescaled BN scale, input range
    const void* wx3_2; const float* scale2_x;
    const unsigned* x2max; float x2bound;
    int x_exact;                                 // fp16 pairs: input values exact in fp16 (integer canvas)
    int mbase;                                   // conv_x6 tiles: first output row of the launch (tail split)
    int dbg;                                     // VdTune::x6_dbg (bits 0-1, timing experiments; 0 in production),
                                                 // bit 2: VdTune::x6_one, bits 3-4: VdTune::x6_halo_dma
    int grp_co, grp_ci;                          // grouped conv (fp32 halo tiles): output channels n read input
                                                 //   channels (n / grp_co) * grp_ci + [0, cin); 0: dense
};

// One fused layer1 bottleneck (block.hip): x [B][H][W][cin] -> y [B][H][W][256],
// weights pre-packed by the runtime (Ctx::make_block) from the per-conv bf16 weights.
struct BlockArgs {
    const void* x; void* y;
    int B, H, W, cin, ds;        // ds: identity = bn(downsample(x)) (cin 64), else x (cin 256)
    int tiles_x, tiles_y;        // 16-wide x 8-high output tiles
    const void* w1;              // conv1 MFMA fragments [4 groups of 16 ch][cin/32 k-steps][64 lanes][8]
    const void* w2;              // conv2 fragments [4][18][64][8]
    const void* w3;              // conv3 fragments [8 groups of 32 ch][2 tiles][2 k-steps][64][8]
    const void* wd;              // downsample fragments [8][2][cin/32][64][8] (ds)
    const float* bn;             // s1 t1 s2 t2 (64 each) s3 t3 sd td (256 each)
    unsigned long long* diag;    // optional: per-stage cycle sums of workgroup 0, wave 0 (tools/convbench)
    int mode;                    // experiments (tools/convbench VD_BLOCK_MODE); 0 in production
    int f16;                     // fp16 plan: fp16 operands / activations (else bf16)
};

// One fused layer1 bottleneck in the fp32 plan (block32.hip): x f32 [B][H][W][cin]
// -> y f32 [B][H][W][256]; weights as fp16 hi / lo planes of the per-conv pair
// packing (row scales folded into the BN scales), per-frame range slots of x / y.
struct Block32Args {
    const void* x; void* y;
    int B, H, W, cin, ds;
    int tiles_x, tiles_y;        // 16-wide x 8-high output tiles
    const void* w1;              // conv1 planes [2][cin/32][64 rows][32] fp16 (LDS image source)
    const void* w2;              // conv2 fragments [4 jn][2 hf][9 taps][2 planes][64 lanes][8] fp16
    const void* w3;              // conv3 fragments [8 waves][2 tiles][2 k-steps][2 planes][64][8] (rows permuted)
    const void* wd;              // downsample fragments, same layout (ds)
    const float* bn;             // s1 h1 s2 h2 (64 each), s3 h3 (256 each), sd hd (256 each, ds)
    const unsigned* xmax;        // x's per-frame max |x| slots (frame 0 of this call)
    unsigned* ymax;              // y's slots (atomic max)
    int xdepth;                  // stage-1 x register sets (option block32_xd: 2, 3, 4)
    int pipe;                    // producer / consumer wave groups on consecutive tiles (option block32_pipe)
    int dbg;                     // timing-only stage skips of the one-group kernel (option block32_dbg; wrong results)
};

// A bottleneck's conv3 (+ identity, ReLU) and the next bottleneck's conv1 in one
// pass (chain.hip): y = relu(bn3(w3 . t2) + res) [M][512], y2 = relu(bn1'(w1 . y)) [M][128].
struct ChainArgs {
    const void* t2; int ld_t2;            // [M][128] bf16
    const void* res; int ld_res;          // identity [M][512]
    const void* w3; int kpad3;            // conv3 weights [>= 512][kpad3] bf16
    const float* sc3; const float* sh3;   // bn3 folded
    const void* w1; int kpad1;            // next conv1 weights [>= 128][kpad1] bf16
    const float* sc1; const float* sh1;   // next bn1 folded
    void* y; int ld_y;                    // block output [M][512]
    void* y2; int ld_y2;                  // next block's t1 [M][128]
    int M;
    int f16;                              // fp16 plan: fp16 operands / activations (else bf16)
};

// fp32 plan (chain32.hip): layer2 conv3 (+ identity, ReLU) and the next conv1 in one pass,
// fp16-pair weights: y = relu(bn3(w3 . t2) + res) [M][512], y2 = relu(bn1'(w1 . y)) [M][128].
struct Chain32Args {
    const void* t2; int ld_t2;            // [M][128] f32
    const void* res; int ld_res;          // identity [M][512] f32
    const void* w3;                       // conv3 planes [>= 512][4 k-steps][2][32] fp16 (conv_x6 wx3)
    const void* w1;                       // next conv1 planes [>= 128][16][2][32], K permuted per 32-step
    const float* sc3; const float* sh3;   // bn3 (scale times the row's 2^-e)
    const float* sc1; const float* sh1;   // next bn1
    void* y; int ld_y;                    // block output [M][512]
    void* y2; int ld_y2;                  // next block's t1 [M][128]
    int M, B, hw;                         // pixels, frames, pixels per frame
    const unsigned* xmax; float xbound;   // t2's per-frame max |x| slots (frame 0 of this call)
    unsigned* ymax; unsigned* y2max;      // y's / y2's slots (atomic max)
    int gpw;                              // 16-pixel groups per wave (layer2: 1 or 2)
};

// Depthwise 3x3 conv (pad 1) + BN + activation, NHWC (dwconv.hip): MobileNetV1 conv_dw.
struct DwConvArgs {
    const void* x; int xh, xw, ldx, xcoff;
    const void* w;                               // [9 taps][c] (dy-major), compute type
    const float* scale; const float* shift;
    void* y; int yh, yw, ldy, ycoff;
    int B, c, stride, act; float slope;
    unsigned* ymax;                              // fp16-pair plan: per-frame max |y| slots, or NULL
};

// RetinaFace stem conv (space-to-depth form) + maxpool in one kernel (stem.hip):
// x = X' [B][xh][xw][16] -> y = pooled [B][ph][pw][64].
struct StemPoolArgs {
    const void* x; int B, xh, xw;
    void* y; int ph, pw;
    const void* wf;              // MFMA fragments [4 groups of 16 ch, pairs permuted][8 k-steps][64 lanes][8]
                                 //   (fp32 plan: [2 planes: hi, lo] of that, fp16; x = X' in fp16, exact)
    const float* scale; const float* shift;
    unsigned* ymax;              // fp32 plan: per-frame max |y| slots of the pooled map
    int f16;                     // fp16 plan (stem_pool_kernel): fp16 canvas, weights and pooled map
};

// Device buffers + parameters for one frame batch's detection post-processing.
enum { POST_FACE = 0, POST_YOLO = 1 };
struct PostArgs {
    int mode;                // POST_FACE / POST_YOLO
    const float* heads[3];   // per level NHWC [B][H][W][hstride] f32
    int hstride;             // face: 32 (0..7 bbox, 8..11 cls, 12..31 landm); yolo: 64 DFL | nc cls (padded)
    int lh[3], lw[3];        // level dims
    int loff[3];             // first anchor index per level
    int strides[3];          // yolo: 8/16/32
    const float* anchors;    // face: [A][4] priors
    int A;                   // anchors per frame
    int B;
    int nc;                  // yolo classes
    float conf;
    double iou;
    int max_det;             // yolo: 300 (0 = unlimited)
    float max_wh;            // yolo class offset (7680)
    uint64_t* cand_keys;     // [B][A] candidate keys
    int* cand_count;         // [B]
    float4* scratch_box;     // [B][A] decoded box by anchor (candidates only)
    int* scratch_cls;        // [B][A] yolo class by anchor
    float4* scratch_nbox;    // [B][A] NMS boxes for large candidate sets
    float* scratch_area;     // [B][A]
    uint64_t* scratch_keys;  // [B][sort_cap]
    uint8_t* scratch_supp;   // [B][A]
    int sort_cap;            // power of two >= A
    int img_h, img_w;        // source frame size (all frames of a call share it)
    float offx, offy, scx, scy;   // face correction (utils_bbox.py:118-132, float32)
    int padx, pady; float inv_gain;  // yolo scale_boxes
    int cap;                 // caller's capacity per frame (out_* may all be NULL)
    int kcap;                // complete keep list capacity per frame (>= any keep count)
    int* k_count;            // [B]          complete keep lists (library-owned; the mosaic's input)
    int* k_xyxy;             // [B][kcap][4]
    float* k_xyxy_f;         // [B][kcap][4]
    float* k_score;          // [B][kcap]
    int* k_label;            // [B][kcap]
    int* out_count;          // [B]
    int* out_xyxy;           // [B][cap][4]
    float* out_xyxy_f;       // [B][cap][4]
    float* out_score;        // [B][cap]
    int* out_label;          // [B][cap]
};

enum { LB_COPY = 0, LB_AREA2 = 1, LB_LINEAR = 2 };

struct LetterboxArgs {
    const uint8_t* src; int n, ih, iw; size_t pitch;
    int oh, ow;            // canvas size
    int nh, nw;            // resized size
    int top, left;         // paste offset
    int mode;
    double scale_x, scale_y;   // 1 / inv_scale (resize.cpp)
    float pad_value;       // canvas fill (128 RetinaFace / 114 YOLO)
    float mean[3];         // subtracted per output channel
    float div;             // divisor after mean (1, or 255 for ultralytics' im /= 255)
    int flip;              // 1: output channel c takes source channel 2-c
    void* out; int cpad; int out_f32;
    int out_f16;           // 16-bit canvas in fp16 (VD_PREC_FP16) instead of bf16
    int s2d;               // 1: space-to-depth canvas for the stride-2 stem (bf16, 16 channels):
                           //    out[Y][X][(py*2+px)*4 + c] = canvas[2Y+py-1][2X+px-1][c], 0 off-canvas,
                           //    Y in [0, oh/2], X in [0, ow/2]
    int gx_k, gx_c;        // set by the launcher (pre.hip): gx_k > 0 when the LB_LINEAR column taps are
                           //    an exact gather, source column gx_k * rx + gx_c with weights (1, 0)
};

// One batch of JPEG frames (jpeg_host.cpp -> jpeg.hip): sparse coefficients per
// block, block order (image, component, block row, block col).
struct JpegArgs {
    int n, h, w, nc, hmax, vmax;
    int bw[3], bh[3], hs[3], vs[3], cblk[3];    // per component: block grid, sampling, first block
    long plane_off[3];
    int blocks_per_image;
    const uint32_t* blk_off;                    // [n * blocks_per_image + 1] into entries
    const uint16_t* quant;                      // [n][3][64] natural order
    const uint32_t* entries;                    // natural index << 16 | int16 quantized value
    uint8_t* planes;                            // [n * blocks_per_image][64] decoded samples
    const int16_t* dense;                       // or (device entropy decode) dense quantized blocks
                                                // [n * blocks_per_image][64] natural order; entries unused
    uint8_t* out; size_t pitch;                 // RGB frames [n][h][pitch]
    int fx[3], fy[3], dw[3], dh[3];             // per component: upsampling factors, downsampled size
                                                // (vd_launch_jpeg fills them)
};

// TERMS = 2 (fp16 pair): each frame's activations are scaled by a power of two so
// their largest magnitude (the producer's per-frame running max, or a static bound
// for the letterboxed canvas) lands in [2^14, 2^15): fp16 never overflows and the
// low term stays normal down to 2^-2 of that. A row (pixel) keeps one scale over
// all of K, so the accumulator is scaled back per row in the epilogue (exact:
// powers of two), and a frame's result does not depend on the rest of its batch.
// Returns the exponent k (operand * 2^k) for frame b.
// the exponent from a frame's max |x| already loaded (act_scale_exp split for prefetching)
__device__ __forceinline__ int act_scale_exp_of(float m) {
    if (!(m > 0.f) || !(m < 3.0e38f)) return 0;
    int e;
    (void)frexpf(m, &e);                              // m < 2^e
    const int k = 15 - e;
    return k < -100 ? -100 : (k > 100 ? 100 : k);
}

__device__ __forceinline__ int act_scale_exp(const ConvArgs& a, int b) {
    const float m = a.xmax ? __uint_as_float(a.xmax[b]) : a.xbound;
    if (!(m > 0.f) || !(m < 3.0e38f)) return 0;
    int e;
    (void)frexpf(m, &e);                              // m < 2^e
    const int k = 15 - e;
    return k < -100 ? -100 : (k > 100 ? 100 : k);
}

// Per-frame running max |y| into the output's slots (non-negative floats order as
// their bit patterns; NaNs are ignored). A lane folds its outputs into (frame, max)
// and flushes on a frame change (rows only ascend, so rarely); at the end the wave
// merges the lanes of its lowest frame into one atomic.
struct AmaxTrack {
    int b = -1;
    float m = 0.f;
    __device__ __forceinline__ void add(unsigned* slot, int fb, float v) {
        if (fb != b) {
            if (b >= 0 && m > 0.f) atomicMax(slot + b, __float_as_uint(m));
            b = fb;
            m = 0.f;
        }
        m = fmaxf(m, v);
    }
    __device__ __forceinline__ void publish(unsigned* slot) {
        int lo = b >= 0 ? b : 0x7fffffff;
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) lo = min(lo, __shfl_xor(lo, o));
        float v = (b == lo) ? m : 0.f;
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
        if ((threadIdx.x & 63) == 0 && lo != 0x7fffffff && v > 0.f) atomicMax(slot + lo, __float_as_uint(v));
        if (b >= 0 && b != lo && m > 0.f) atomicMax(slot + b, __float_as_uint(m));
    }
};

// Workgroup-local form for the conv kernels (one launch touches every frame, so
// per-lane global atomics would serialise on 64 addresses): every lane of a wave
// calls amax_lds_add convergently with its output's frame (-1: none) and max |y|;
// the wave merges its lowest frame into one LDS atomic (other frames: rare, per
// lane), and amax_lds_flush moves the workgroup's nonzero slots to global.
__device__ __forceinline__ void amax_lds_add(unsigned* s, int fb, float v) {
    int lo = fb >= 0 ? fb : 0x7fffffff;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) lo = min(lo, __shfl_xor(lo, o));
    if (lo == 0x7fffffff) return;                     // wave-uniform
    float m = (fb == lo) ? v : 0.f;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    if ((threadIdx.x & 63) == 0 && m > 0.f) atomicMax(s + lo, __float_as_uint(m));
    if (fb >= 0 && fb != lo && v > 0.f) atomicMax(s + fb, __float_as_uint(v));
}

__device__ __forceinline__ void amax_lds_flush(const unsigned* s, unsigned* g, int nframes) {
    for (int f = threadIdx.x; f < nframes; f += blockDim.x)
        if (s[f]) atomicMax(g + f, s[f]);
}

// Device entropy decode (jpeg_dec.hip). JLds: one Huffman table set as the kernels
// hold it in LDS (jpeg_host.cpp build_huff tables): 11-bit lookahead (len << 8 | sym)
// for dc0 dc1 ac0 ac1, the AC fast path (len | run << 8 | (u16)value << 16; run 64 =
// EOB, 16 = ZRL), and the canonical slow path.
struct JLds {
    uint16_t look[4][2048];
    uint32_t fast[2][2048];
    uint32_t fastdc[2][2048];                   // DC code + extra bits in one lookup (len | diff << 16)
    int32_t maxcode[4][18];
    int32_t valoff[4][17];
    uint8_t vals[4][256];
};
struct JdecLaunch {
    int stage;                     // 0 prep, 1 sync pass, 2 scan, 3 write
    int pass, nwg;
    const int* wg_frame; const uint32_t* wg_chunk;   // workgroup -> (frame, first chunk)
    const uint8_t* bytes; const uint32_t* seg_off; const uint32_t* seg_len; const uint32_t* chunk0;
    const uint8_t* tab_of; const JLds* tabs;
    int n, chunk_bytes, bpm;
    int ucomp[6], udc[6], uac[6], ubx[6], uby[6];
    int mcux, total_blocks;
    int cblk[3], bw[3], hs[3], vs[3];
    int blocks_per_image;
    uint32_t* D; uint32_t* S; uint8_t* Su;
    uint32_t* Epos[2]; uint8_t* Eu[2];
    uint32_t* nblk; int* dcs; uint32_t* base; int* dcoff;
    int16_t* dense;
    int* flags;
    int R; uint32_t* Lpos[2]; uint8_t* Lu[2]; int* Ldc[2]; uint8_t* Lcnt[2]; uint8_t* Lsel; uint32_t* own;
};
hipError_t vd_launch_jdec(const JdecLaunch& L, hipStream_t s);

// One batch of RGB frames -> quantized coefficient blocks (jpeg_enc.hip -> jpeg_enc.cpp).
struct JpegEncArgs {
    const uint8_t* src; size_t pitch; int n, h, w;
    int hl, vl;                                 // luma sampling factors (chroma 1x1)
    int bw[3], bh[3];                           // blocks per component (width/height_in_blocks)
    long cblk[3], blocks_per_frame;             // first block of each component within a frame
    const uint16_t* recip; const uint16_t* corr; const uint8_t* shift;   // [2 tables][64], natural order
    int16_t* coef;                              // [n][blocks_per_frame][64] natural order
};

// Device entropy stage (jpeg_enc.hip, after jpeg_fdct_kernel): one thread per
// scan unit (a block in MCU order, dummy blocks included) sizes, then writes, its
// Huffman code; a per-frame scan gives the bit offsets; a stuffing pass emits the
// entropy-coded segment with 0xFF 0x00 and the 1-bit padding.
struct JpegHuffArgs {
    const int16_t* coef; long blocks_per_frame; int n;
    int hl, vl, bw[3], bh[3]; long cblk[3];
    int mcux, units;                            // MCUs per row; scan units per frame
    const uint16_t* code; const uint8_t* size;  // [4][256]: DC luma, DC chroma, AC luma, AC chroma
    unsigned* bits;                             // [n][units] code length, then exclusive bit offset
    unsigned* total;                            // [n] bits per frame
    unsigned* words; long wcap;                 // [n][wcap] MSB-first bit buffer (zeroed)
    uint8_t* seg; long segcap; unsigned* segsize;   // stuffed segments packed frame after frame; lengths
    unsigned* ffcnt; int nchunk;                // [n][nchunk] 0xFF bytes per 4-KB chunk, then output offsets
    unsigned long long* segbase;                // [n + 1] frame offsets in seg (exclusive scan; [n] = total)
};

// ---- kernel launchers (one translation unit each) ----
hipError_t vd_launch_jpeg_fdct(const JpegEncArgs& a, hipStream_t s);
hipError_t vd_launch_jpeg_huff(const JpegHuffArgs& a, hipStream_t s);          // codes -> words, bit totals
hipError_t vd_launch_jpeg_stuff(const JpegHuffArgs& a, hipStream_t s);         // words -> packed segments
hipError_t vd_launch_amax_merge(unsigned* dst, const unsigned* src, int n, hipStream_t s);
bool vd_conv1x1_stream_ok(const ConvArgs& a);
bool vd_conv_big_ok(const ConvArgs& a);
hipError_t vd_launch_conv_big(const ConvArgs& a, hipStream_t s);
hipError_t vd_launch_conv1x1_stream(const ConvArgs& a, hipStream_t s);
bool vd_conv_taps_ok(const ConvArgs& a);
bool vd_conv1x1_dual_ok(const ConvArgs& a);
hipError_t vd_launch_conv_taps(const ConvArgs& a, hipStream_t s);
hipError_t vd_launch_conv(const ConvArgs& a, bool f32, hipStream_t s);
bool vd_conv_x6_ok(const ConvArgs& a);
bool vd_conv1x1_x6_dual_ok(const ConvArgs& a);
hipError_t vd_launch_conv_x6(const ConvArgs& a, hipStream_t s);
void vd_pack_x6(const float* w, int npad, int kpad, uint16_t* out);   // host: f32 [npad][kpad] -> split planes
void vd_pack_x3h(const float* w, int npad, int kpad, uint16_t* out, float* row_inv);   // ... fp16 pairs
bool vd_block_ok(int cin, bool ds, int h, int w);
bool vd_block32_ok(int cin, bool ds, int h, int w);
hipError_t vd_launch_block32(const Block32Args& a, hipStream_t s);
bool vd_stem_pool_ok(int xh, int xw, int ph, int pw);
hipError_t vd_launch_dwconv(const DwConvArgs& a, bool f32, bool f16, hipStream_t s);
hipError_t vd_launch_stem_pool(const StemPoolArgs& a, hipStream_t s);
hipError_t vd_launch_stem_pool32(const StemPoolArgs& a, hipStream_t s);   // fp16-pair plan, f32 pooled map
hipError_t vd_launch_block(const BlockArgs& a, hipStream_t s);
bool vd_chain_ok(int cmid, int cout, int kpad3, int kpad1, int ld_t2, int ld_res, int ld_y, int ld_y2, long M);
hipError_t vd_launch_chain(const ChainArgs& a, hipStream_t s);
bool vd_chain32_ok(int cmid, int cout, int kpad3, int kpad1, int ld_t2, int ld_res, int ld_y, int ld_y2, long M,
                   int frames);
hipError_t vd_launch_chain32(const Chain32Args& a, hipStream_t s);
hipError_t vd_launch_letterbox(const LetterboxArgs& a, hipStream_t s);
bool vd_letterbox_pair_ok(const LetterboxArgs& a, const LetterboxArgs& b);
hipError_t vd_launch_letterbox_pair(const LetterboxArgs& a, const LetterboxArgs& b, hipStream_t s);
hipError_t vd_launch_maxpool(bool f32, bool f16, const void* x, int n, int xh, int xw, int ldx, int xcoff,
                             void* y, int yh, int yw, int ldy, int ycoff, int c, int k, int st, int p,
                             hipStream_t s);
hipError_t vd_launch_upsample2x(bool f32, const void* x, int n, int xh, int xw, int ldx, int xcoff,
                                void* y, int ldy, int ycoff, int c, hipStream_t s);
hipError_t vd_launch_post(const PostArgs& p, hipStream_t s);
hipError_t vd_launch_jpeg(const JpegArgs& a, hipStream_t s);
hipError_t vd_launch_mosaic(const uint8_t* in, uint8_t* out, int n, int h, int w, size_t pitch,
                            const int* cnt0, const int* xy0, int cap0,
                            const int* cnt1, const int* xy1, int cap1, int level, void* table,
                            int stages, int map_on, int cell_blocks, hipStream_t s);   // stages: 1 = cell table, 2 = output pass, 4 = copy
size_t vd_mosaic_table_bytes(int n, int tcap);

#define VD_CHECK_HIP(expr)                                                     \
    do {                                                                       \
        hipError_t _e = (expr);                                                \
        if (_e != hipSuccess) {                                                \
            vd_set_error(VD_ERR_HIP, "%s:%d %s -> %s", __FILE__, __LINE__,      \
                         #expr, hipGetErrorString(_e));                        \
            return VD_ERR_HIP;                                                 \
        }                                                                      \
    } while (0)

int vd_set_error(int code, const char* fmt, ...);
