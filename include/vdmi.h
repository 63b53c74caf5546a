/*
 * vdmi.h — C-ABI of libvdmi.so, the MI355X-native detect-and-blur hot path.
 *
 * This is the drop-in boundary for the per-frame path of the reference
 * (xdu-Liu-learn/Video-desensitization). Each entry point names the reference
 * interface it replaces (paths relative to the reference repository root):
 *
 *   vd_create / vd_load_weights  <- Retinaface.__init__/generate   detect_face/face.py:29-60
 *                                   YOLO(plate_model_path).cuda()   combine_detect.py:872
 *   vd_detect                    <- Retinaface.detect_images        detect_face/face.py:120-150
 *                                   (preprocess :65-88, net :133, postprocess :93-115,
 *                                    scaling :139-146) + int() at combine_detect.py:243
 *   vd_detect_plates             <- plate_detector(batch, verbose=False, conf=0.5)
 *                                                                    combine_detect.py:217
 *   vd_mosaic                    <- mosaic_rectangle_region_single  combine_detect.py:138-161,
 *                                   applied per box in order at     combine_detect.py:246-249
 *   vd_process                   <- the per-batch body of batch_process_images
 *                                                                    combine_detect.py:214-251
 *   vd_jpeg_decode / vd_jpeg_info <- cv2.imread(path) + cvtColor(BGR2RGB) of the ffmpeg-split
 *                                   frames                         combine_detect.py:167-172,
 *                                   (frames from convert_video_to_frames :279-476)
 *   vd_read_boxes                <- the complete per-frame box lists the reference's
 *                                   loop iterates (combine_detect.py:241-249), past any cap
 *   vd_sync / vd_last_error / vd_destroy: runtime plumbing (no reference equivalent;
 *                                   errors map to the reference's drop-the-batch
 *                                   behaviour at combine_detect.py:226-228 in the
 *                                   Python wrapper).
 *
 * Conventions: plain pointers and sizes only. Frames are uint8 RGB, HxWx3,
 * row pitch in bytes, frame i at base + i*h*pitch. `where` says whether a
 * pointer is host (VD_HOST) or device (VD_DEVICE) memory of the context's GPU.
 * The caller owns frames and box arrays; the library owns weights, device
 * workspace and its stream. No pointer is retained past a call. Calls are
 * asynchronous on the context stream only when every pointer is VD_DEVICE;
 * otherwise they return after results are in the caller's host memory.
 * Return value: VD_OK (0) or a negative VD_ERR_*; vd_last_error() gives a
 * thread-local message. Calls on one context are serialised by a mutex;
 * different contexts are independent (one per device/stream).
 */
#ifndef VDMI_H
#define VDMI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VDMI_ABI_VERSION 2   /* 2: complete keep lists (count may exceed cap, vd_read_boxes) */

#define VD_OK            0
#define VD_ERR_ARG      -1   /* bad argument / shape */
#define VD_ERR_HIP      -2   /* HIP runtime error */
#define VD_ERR_CAPACITY -3   /* vd_mosaic: a host box list's count exceeds its cap */
#define VD_ERR_WEIGHTS  -4   /* weight blob missing a tensor / wrong shape */
#define VD_ERR_STATE    -5   /* call out of order (e.g. detect before weights) */
#define VD_ERR_NOMEM    -6   /* device allocation failed */

#define VD_HOST   0
#define VD_DEVICE 1

#define VD_PREC_BF16 0       /* bf16 operands, f32 accumulate (performance mode) */
#define VD_PREC_FP32 1       /* f32 operands and activations (parity mode): operands
                              * scaled by powers of two (per frame / per output
                              * channel) and split into fp16 pairs, 3 products on
                              * the f16 matrix cores, f32 accumulate; option
                              * f32_split=1: exact 3-term bf16 split (6 products),
                              * 0: exact-f32 MFMA */
#define VD_PREC_FP16 2       /* fp16 operands, f32 accumulate on                  *
                              * v_mfma_f32_16x16x32_f16; the bf16 plan's fused     *
                              * kernels (stem + pool, layer1 blocks, layer2        *
                              * chains, phased 256x256) templated on the 16-bit type */

#define VD_NET_RETINAFACE 0  /* detect_face/retinaface.py, cfg_re50 */
#define VD_NET_YOLOV8N    1  /* ultralytics YOLOv8n plate detector [ext] */

#define VD_WEIGHTS_VDW1   1  /* "VDW1" named-tensor container, see DESIGN.md */

/* vd_mosaic modes */
#define VD_MOSAIC_OUT_OF_PLACE 0   /* out = in with boxes applied (reference new-array semantics) */

/* vd_process flags */
#define VD_PROC_FACES        1     /* run the RetinaFace branch */
#define VD_PROC_PLATES       2     /* run the YOLOv8n branch (forward + NMS) */
#define VD_PROC_MOSAIC       4     /* write mosaicked frames to `out` */
#define VD_PROC_MOSAIC_PLATES 8    /* "intended mode": mosaic plate boxes too. Without it
                                      plate boxes are discarded like the reference
                                      (combine_detect.py:239 always yields []). */

typedef struct vd_ctx vd_ctx;

typedef struct vd_cfg {
    int32_t input_h, input_w;      /* RetinaFace net input; combine_detect.py:860 uses 640x640 */
    int32_t max_batch;             /* frames per call (config.ini:35 batch_size = 64) */
    int32_t max_frame_h, max_frame_w;
    int32_t precision;             /* VD_PREC_* */
    int32_t max_boxes;             /* per-frame capacity of the NMS output list */
    float   confidence;            /* face score threshold, inclusive (utils_bbox.py:116) */
    double  nms_iou;               /* face NMS IoU (combine_detect.py:862 -> 0.4) */
    int32_t mosaic_level;          /* combine_detect.py:249 -> 8 */
    int32_t plate_imgsz;           /* ultralytics imgsz (640) */
    int32_t plate_nc;              /* plate model classes */
    float   plate_conf;            /* combine_detect.py:217 conf=0.5 */
    double  plate_iou;             /* ultralytics default 0.7 [ext] */
    int32_t plate_max_det;         /* ultralytics default 300 [ext] */
    int32_t reserved[8];
} vd_cfg;

/* Per-frame box lists, caller-allocated. Frame f's boxes live at
 * [f*cap, f*cap + min(count[f], cap)). count[f] is always the COMPLETE keep count
 * and may exceed cap: the arrays then hold the first cap boxes (NMS order), the
 * call still succeeds, vd_read_boxes hands out the complete lists, and the
 * mosaic of vd_process always covers every kept box (the reference blurs every
 * box, combine_detect.py:241-249). A NULL vd_boxes* skips the caller copy. */
typedef struct vd_boxes {
    int32_t  cap;
    int32_t  where;     /* VD_HOST or VD_DEVICE for every array below */
    int32_t* count;     /* [n]            */
    int32_t* xyxy;      /* [n][cap][4]    int() of the source-pixel box (combine_detect.py:243) */
    float*   xyxy_f;    /* [n][cap][4]    float32 source-pixel box before int(); may be NULL */
    float*   score;     /* [n][cap]       may be NULL */
    int32_t* label;     /* [n][cap]       anchor index (faces) / class id (plates); may be NULL */
} vd_boxes;

int         vd_default_cfg(vd_cfg* cfg);
int         vd_abi_version(void);
const char* vd_last_error(void);

int   vd_create(const vd_cfg* cfg, int device, vd_ctx** out);
int   vd_destroy(vd_ctx* ctx);
int   vd_load_weights(vd_ctx* ctx, int net, const void* blob, size_t bytes, int fmt);
int   vd_set_stream(vd_ctx* ctx, void* hip_stream);   /* NULL -> library-owned stream */
/* Kernel-selection switches (A/B measurement, tests that force a kernel form onto
 * small shapes); the defaults are the production plan. Plan switches (block_fuse,
 * chain, stem_pool, ssh_fuse, plate_s2d, f32_split) apply to weights loaded afterwards, the
 * rest to the next launch. Names: conv_stream conv_stream512 conv_dual conv_taps
 * conv_n192 conv_small conv_big conv_big_kmin stream_ntt lb_pair mosaic_map
 * block_fuse chain stem_pool ssh_fuse plate_s2d f32_split x6_small_k x6_small_tiles x6_stream
 * x6_small_k2 x6_bn256 x6_exact x6_stream256 plate_stage jenc_gpu (the full list:
 * runtime.cpp vd_set_option).
 * VD_ERR_ARG for unknown names. */
int   vd_set_option(vd_ctx* ctx, const char* name, int value);
/* Test / profiling only: timing experiments that skip work and give WRONG results
 * while set ("x6_dbg": conv epilogues, "block32_dbg": layer1 block stages). They are
 * not vd_set_option names (that call refuses them). VD_ERR_ARG for unknown names. */
int   vdt_set_debug(vd_ctx* ctx, const char* name, int value);
void* vd_get_stream(vd_ctx* ctx);
int   vd_sync(vd_ctx* ctx);

int vd_detect(vd_ctx* ctx, const uint8_t* frames, int n, int h, int w, size_t pitch,
              int where, vd_boxes* faces);
int vd_detect_plates(vd_ctx* ctx, const uint8_t* frames, int n, int h, int w, size_t pitch,
                     int where, vd_boxes* plates);
/* Mosaic of caller box lists; host lists with count[f] > cap are refused
 * (VD_ERR_CAPACITY: boxes the caller does not hold would go unblurred).
 * Out of place only, as the reference blurs a copy (combine_detect.py:142):
 * `out` equal to `in`, or (VD_DEVICE) any overlap of the two n*h*pitch ranges, is
 * VD_ERR_ARG. vd_process with VD_PROC_MOSAIC and VD_DEVICE frames refuses
 * overlapping `in` / `out` the same way (its one-launch output pass gathers cell
 * colours from `in` while other workgroups write `out`); VD_HOST frames are staged
 * in separate device buffers, so host in == out is allowed there. */
int vd_mosaic(vd_ctx* ctx, const uint8_t* in, uint8_t* out, int n, int h, int w, size_t pitch,
              int where, const vd_boxes* boxes, int level, int mode);
int vd_process(vd_ctx* ctx, const uint8_t* in, uint8_t* out, int n, int h, int w, size_t pitch,
               int where, int flags, vd_boxes* faces, vd_boxes* plates);
/* Baseline JPEG frames -> RGB frames: the frame read of the reference's loop
 * (cv2.imread + BGR->RGB of the ffmpeg-split frames, combine_detect.py:167-172),
 * libjpeg-turbo's default decode (ISLOW IDCT, fancy upsampling, table YCbCr->RGB),
 * bit-identical. data[i] / sizes[i]: n host JPEG buffers, all h x w with one
 * component layout (1 or 3 components, 1x1 / 2x1 / 2x2 sampling; no progressive /
 * arithmetic coding). Headers parsed and scan segments staged on host threads; the
 * entropy decode runs on the device (chunked speculative Huffman decode with
 * resynchronisation passes; option jdec_gpu=0: host Huffman threads, same pixels),
 * then dequantize + IDCT + upsample + colour in HIP kernels writing `out`
 * (VD_DEVICE: queued on the context stream, the frames feed vd_process directly;
 * VD_HOST: returns when `out` is filled). */
int vd_jpeg_decode(vd_ctx* ctx, const uint8_t* const* data, const size_t* sizes, int n, uint8_t* out,
                   int h, int w, size_t pitch, int where);
int vd_jpeg_info(const uint8_t* data, size_t size, int* h, int* w, int* comps);
/* RGB frames -> baseline JFIF: the frame write of the reference's loop (cv2.imwrite
 * of the processed frames, combine_detect.py:174-180, :259-262; cv2's defaults are
 * quality 95, 4:2:0), libjpeg-turbo's compressor with its defaults bit-identical
 * (Pillow Image.save(..., quality, subsampling) bytes). frames: n frames h x w x 3
 * RGB at `where`; subsampling 0 = 4:4:4, 1 = 4:2:2, 2 = 4:2:0. Colour conversion,
 * downsampling, ISLOW FDCT and quantisation in a HIP kernel; Huffman coding and 0xFF
 * stuffing in HIP kernels (option jenc_gpu=0: on host threads, same bytes); frames
 * up to 2,000,000 scan blocks (8K). Frame i goes to out + i * cap, its length to sizes[i]; VD_ERR_CAPACITY
 * if a frame needs more than cap bytes -- with the device coder sizes[i] then holds an
 * upper bound of frame i's length (re-size and call again), with host threads 0.
 * Returns when every frame is written. */
int vd_jpeg_encode(vd_ctx* ctx, const uint8_t* frames, int n, int h, int w, size_t pitch, int where,
                   int quality, int subsampling, uint8_t* out, size_t cap, size_t* sizes);
/* The complete keep lists of the last vd_detect / vd_detect_plates / vd_process
 * call on this context for frames [0, n) of `net` (VD_NET_*), into `out`
 * (min(count, out->cap) boxes per frame; count = complete count). Ordered on the
 * context stream after that call; host targets return when the copy is done. */
int vd_read_boxes(vd_ctx* ctx, int net, int n, vd_boxes* out);

/* ---- instrumentation (bench / profiling) ---------------------------------- */
/* When enabled, every launch of kernel family `fam` is bracketed by HIP events
 * on the context stream; vd_timing_read returns the summed duration (ms), the
 * launch count and the summed algorithmic work (FLOP or bytes) since the last
 * reset. Families: 0 = RetinaFace conv (implicit GEMM / streaming 1x1), 1 = mosaic
 * output pass, 2 = letterbox, 3 = post (decode/NMS), 4 = other, 5 = YOLOv8n plate
 * conv, 6 = mosaic cell table (box prep + walked cell colours). */
int vd_timing_enable(vd_ctx* ctx, int on);
int vd_timing_reset(vd_ctx* ctx);
int vd_timing_read(vd_ctx* ctx, int fam, double* ms, int64_t* launches, double* work);

/* ---- test hooks (parity tests call these; same kernels as the product path) -- */
/* Letterboxed RetinaFace input, NHWC with cpad channels (f32 regardless of precision). */
int vdt_letterbox(vd_ctx* ctx, const uint8_t* frames, int n, int h, int w, size_t pitch,
                  int where, float* out_nhwc, int cpad);
/* Raw head outputs after the forward, host f32: loc [n][A][4], conf logits [n][A][2],
 * landm [n][A][10], A = number of anchors. */
int vdt_forward_heads(vd_ctx* ctx, const uint8_t* frames, int n, int h, int w, size_t pitch,
                      int where, float* loc, float* conf, float* landm);
/* Post-processing only (decode, score, threshold, NMS, correction, int()) on
 * caller-provided host head outputs; img_hw = [n][2] source sizes. */
int vdt_postprocess(vd_ctx* ctx, const float* loc, const float* conf, int n,
                    const int32_t* img_hw, vd_boxes* faces);
/* One convolution through the product conv kernel (host f32 NHWC in/out,
 * weights [cout][kh][kw][cin] f32, BN as per-channel scale/shift, act 0=none
 * 1=relu 2=leaky(slope) 3=silu; res (optional, NHWC [n][oh][ow][cout]) added
 * before the activation when res_mode=1, after it when res_mode=2). */
int vdt_conv2d(vd_ctx* ctx, const float* x, int n, int h, int w, int cin,
               const float* wgt, int cout, int kh, int kw, int stride, int pad,
               const float* scale, const float* shift, int act, float slope,
               const float* res, int res_mode, float* y, int* oh, int* ow);
/* One ResNet layer1 bottleneck on host f32 NHWC x [n][h][w][cin] -> y [n][h][w][256]
 * (bf16 context): conv1 1x1 cin->64, conv2 3x3 64->64 pad 1, conv3 1x1 64->256, each
 * OIHW weights + BN as bn = [scale[cout] | shift[cout]]; ReLU after each, the residual
 * (x, or bn(downsample(x)) when wd != NULL, cin 64) added before the last ReLU.
 * fused = 1: the one-kernel fused block (block.hip); 0: the conv-by-conv chain. */
int vdt_bottleneck(vd_ctx* ctx, const float* x, int n, int h, int w, int cin,
                   const float* w1, const float* bn1, const float* w2, const float* bn2,
                   const float* w3, const float* bn3, const float* wd, const float* bnd,
                   int fused, float* y);
/* Raw YOLO Detect outputs [n][64+nc][A] (per-side DFL logits | class logits),
 * host f32, anchors in level -> y -> x order at the letterboxed canvas; *anchors
 * receives A. `out` may be NULL to query A. */
/* JPEG host entropy stage alone (no GPU): quantized coefficients [nblocks][64]
 * (natural order; blocks by component, block row, block col); out may be NULL to
 * query nblocks. */
int vdt_jpeg_coefficients(const uint8_t* data, size_t size, int16_t* out, size_t cap_blocks, int* nblocks);
int vdt_plate_raw(vd_ctx* ctx, const uint8_t* frames, int n, int h, int w, size_t pitch,
                  int where, float* out, int* anchors);
/* ---- .record container I/O (host; replaces foreign/recordDeal.so) ------------
 * vd_record_extract_h265: every *.record* file of record_dir (sorted; CyberRT
 * segments) -> <out_dir>/hevcs/<camera>.h265 per camera topic
 * /drivers/camera/<camera>/compressed/image: the CompressedImage data of its
 * messages from the first key frame on, concatenated (replaces
 * recordDeal.read_record2h265_all, combine_detect.py:839).
 * vd_record_repack_h265: the same records rewritten into out_dir with each
 * extracted message's data replaced by the matching access unit of
 * <videos_dir>/<camera>_processed.h265 (or _processed.hevc, processed_<camera>.h265:
 * the desensitised stream, named as combine_detect.py:658 names it; the un-suffixed
 * <camera>.h265 is the extract step's ORIGINAL stream and is refused); everything else
 * carried over, positions and sizes recomputed (replaces
 * recordDeal.write_allH265_record_all, combine_detect.py:958). Uncompressed
 * records only. */
int vd_record_extract_h265(const char* record_dir, const char* out_dir, int* topics_written);
int vd_record_repack_h265(const char* record_dir, const char* videos_dir, const char* out_dir, int* records_written);

/* The last vd_jpeg_decode's device entropy stage: synchronisation passes run (pass 0
 * included; 0 when the host entropy stage ran). */
int vdt_jdec_stats(vd_ctx* ctx, int* passes);

#ifdef __cplusplus
}
#endif
#endif /* VDMI_H */
