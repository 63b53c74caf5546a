// post.hip — detection post-processing on the GPU, bit-exact with the oracle.
//
// Faces: replaces Retinaface.postprocess (detect_face/face.py:93-115) + the host
// scaling loop (face.py:136-148) + int() (combine_detect.py:243):
//   softmax score        retinaface.py:147           (vd_expf, float32 ops)
//   threshold >= conf    utils_bbox.py:115-116
//   decode               utils_bbox.py:49-59         (reference op order, no FMA)
//   batched_nms          utils_bbox.py:121-127 -> torchvision nms [ext]:
//                        stable descending sort, IoU in float32, '>' vs double
//   correct boxes        utils_bbox.py:12-43 (float32 tensors)
//   x [w,h,w,h]          face.py:144-145 (float32 numpy)
//   int()                combine_detect.py:243 (truncation toward zero)
// Plates: the ultralytics predict post-processing of the call at
// combine_detect.py:217 [ext, version unpinned]: DFL decode + dist2bbox,
// sigmoid class scores, conf > 0.5, class-offset NMS at IoU 0.7, max_det 300,
// scale_boxes + clip.
//
// Kernels per batch:
//  *_candidates_kernel  one thread per anchor: score + threshold; survivors get a
//    64-bit key (~score_bits, anchor) -- an ascending sort of the keys is the
//    stable descending-score order torchvision's nms uses -- and their decoded
//    box in a per-anchor scratch.
//  nms_kernel  one 1024-thread workgroup per frame: bitonic sort of the keys,
//    gather of the survivors' boxes, greedy NMS in chunks of 64 (wave 0 resolves
//    a chunk with a 64x64 IoU bitmask and a scalar readlane sweep; then all 16
//    waves suppress later candidates against the chunk's kept boxes; the result
//    is exactly the sequential greedy keep list), then the net's output
//    transform. Up to LDS_CAND candidates live in LDS, more in global scratch.
#include "vd_common.h"
#include "vd_math.h"

namespace {

constexpr int NMS_THREADS = 1024;
constexpr int LDS_CAND = 2048;

__device__ __forceinline__ int level_of(const PostArgs& p, int a) {
    return a >= p.loff[2] ? 2 : (a >= p.loff[1] ? 1 : 0);
}

// ---------------------------------------------------------------- faces (K1)
__global__ __launch_bounds__(256) void face_candidates_kernel(PostArgs p) {
    const int a = blockIdx.x * 256 + threadIdx.x;
    const int b = blockIdx.y;
    if (a >= p.A) return;
    const int l = level_of(p, a);
    const int local = a - p.loff[l];
    const int pix = local >> 1, k = local & 1;
    const float* h = p.heads[l] + ((size_t)b * p.lh[l] * p.lw[l] + pix) * p.hstride;
    const float c0 = h[8 + 2 * k], c1 = h[9 + 2 * k];
    const float m = c0 > c1 ? c0 : c1;
    const float e0 = vd_expf(VD_FSUB(c0, m));
    const float e1 = vd_expf(VD_FSUB(c1, m));
    const float s = VD_FDIV(e1, VD_FADD(e0, e1));
    if (!(s >= p.conf)) return;
    // decode (utils_bbox.py:49-59)
    const float* lo = h + 4 * k;
    const float4 pr = *(const float4*)(p.anchors + 4 * (size_t)a);
    const float v0 = 0.1f, v1 = 0.2f;
    const float cx = VD_FADD(pr.x, VD_FMUL(VD_FMUL(lo[0], v0), pr.z));
    const float cy = VD_FADD(pr.y, VD_FMUL(VD_FMUL(lo[1], v0), pr.w));
    const float w = VD_FMUL(pr.z, vd_expf(VD_FMUL(lo[2], v1)));
    const float hh = VD_FMUL(pr.w, vd_expf(VD_FMUL(lo[3], v1)));
    const float x1 = VD_FSUB(cx, VD_FDIV(w, 2.0f));
    const float y1 = VD_FSUB(cy, VD_FDIV(hh, 2.0f));
    p.scratch_box[(size_t)b * p.A + a] = make_float4(x1, y1, VD_FADD(w, x1), VD_FADD(hh, y1));
    const int pos = atomicAdd(&p.cand_count[b], 1);
    p.cand_keys[(size_t)b * p.A + pos] = ((uint64_t)(0xFFFFFFFFu - __float_as_uint(s)) << 32) | (uint32_t)a;
}

// ---------------------------------------------------------------- plates (K1)
// ultralytics Detect._inference + non_max_suppression candidate filter [ext]
__global__ __launch_bounds__(256) void yolo_candidates_kernel(PostArgs p) {
    const int a = blockIdx.x * 256 + threadIdx.x;
    const int b = blockIdx.y;
    if (a >= p.A) return;
    const int l = level_of(p, a);
    const int pix = a - p.loff[l];
    const int gy = pix / p.lw[l], gx = pix - gy * p.lw[l];
    const float* h = p.heads[l] + ((size_t)b * p.lh[l] * p.lw[l] + pix) * p.hstride;
    // class scores: sigmoid, max over classes (first index on ties)
    float best = -1.f;
    int cls = 0;
    for (int c = 0; c < p.nc; ++c) {
        const float sg = VD_FDIV(1.0f, VD_FADD(1.0f, vd_expf(-h[64 + c])));
        if (sg > best) { best = sg; cls = c; }
    }
    if (!(best > p.conf)) return;            // xc = amax > conf_thres (strict)
    // DFL: softmax over 16 bins per side, expectation with weights 0..15
    float d[4];
    for (int sd = 0; sd < 4; ++sd) {
        const float* q = h + sd * 16;
        float mx = q[0];
        for (int i = 1; i < 16; ++i) mx = q[i] > mx ? q[i] : mx;
        float e[16], sum = 0.f;
        for (int i = 0; i < 16; ++i) { e[i] = vd_expf(VD_FSUB(q[i], mx)); sum = VD_FADD(sum, e[i]); }
        float acc = 0.f;
        for (int i = 0; i < 16; ++i) acc = VD_FADD(acc, VD_FMUL(VD_FDIV(e[i], sum), (float)i));
        d[sd] = acc;
    }
    const float ax = VD_FADD((float)gx, 0.5f), ay = VD_FADD((float)gy, 0.5f);
    const float st = (float)p.strides[l];
    // dist2bbox(xywh=True) * stride, then xywh2xyxy
    const float x1 = VD_FSUB(ax, d[0]), y1 = VD_FSUB(ay, d[1]);
    const float x2 = VD_FADD(ax, d[2]), y2 = VD_FADD(ay, d[3]);
    const float cx = VD_FMUL(VD_FDIV(VD_FADD(x1, x2), 2.0f), st);
    const float cy = VD_FMUL(VD_FDIV(VD_FADD(y1, y2), 2.0f), st);
    const float bw = VD_FMUL(VD_FSUB(x2, x1), st), bh = VD_FMUL(VD_FSUB(y2, y1), st);
    const float hw = VD_FDIV(bw, 2.0f), hh = VD_FDIV(bh, 2.0f);
    p.scratch_box[(size_t)b * p.A + a] = make_float4(VD_FSUB(cx, hw), VD_FSUB(cy, hh), VD_FADD(cx, hw), VD_FADD(cy, hh));
    p.scratch_cls[(size_t)b * p.A + a] = cls;
    const int pos = atomicAdd(&p.cand_count[b], 1);
    p.cand_keys[(size_t)b * p.A + pos] = ((uint64_t)(0xFFFFFFFFu - __float_as_uint(best)) << 32) | (uint32_t)a;
}

__device__ __forceinline__ int trunc_i32(float v) {
    // int(x) of a Python float; values beyond int32 are clamped (the mosaic clips
    // to the frame first, combine_detect.py:145-148, so the output is unchanged).
    if (!(v == v)) return 0;
    if (v >= 2147483520.0f) return 2147483647;
    if (v <= -2147483648.0f) return (-2147483647 - 1);
    return (int)v;   // truncation toward zero
}

__device__ __forceinline__ float clampf(float v, float lo, float hi) { return v < lo ? lo : (v > hi ? hi : v); }

// Kept box `pos` of frame b: always into the library's complete keep list (what the
// mosaic reads), and into the caller's arrays while pos < cap.
__device__ void emit(const PostArgs& p, int b, int pos, float4 bx, uint64_t key) {
    const size_t k = (size_t)b * p.kcap + pos;
    float X1, Y1, X2, Y2;
    const int a = (int)(key & 0xFFFFFFFFu);
    if (p.mode == POST_FACE) {
        // (box - offset) * scale, then * [w, h, w, h]  (utils_bbox.py:137, face.py:145)
        const float iw = (float)p.img_w, ih = (float)p.img_h;
        X1 = VD_FMUL(VD_FMUL(VD_FSUB(bx.x, p.offx), p.scx), iw);
        Y1 = VD_FMUL(VD_FMUL(VD_FSUB(bx.y, p.offy), p.scy), ih);
        X2 = VD_FMUL(VD_FMUL(VD_FSUB(bx.z, p.offx), p.scx), iw);
        Y2 = VD_FMUL(VD_FMUL(VD_FSUB(bx.w, p.offy), p.scy), ih);
    } else {
        // scale_boxes: (box - pad) * (1/gain), clip to the source frame [ext]
        X1 = clampf(VD_FMUL(VD_FSUB(bx.x, (float)p.padx), p.inv_gain), 0.f, (float)p.img_w);
        Y1 = clampf(VD_FMUL(VD_FSUB(bx.y, (float)p.pady), p.inv_gain), 0.f, (float)p.img_h);
        X2 = clampf(VD_FMUL(VD_FSUB(bx.z, (float)p.padx), p.inv_gain), 0.f, (float)p.img_w);
        Y2 = clampf(VD_FMUL(VD_FSUB(bx.w, (float)p.pady), p.inv_gain), 0.f, (float)p.img_h);
    }
    const int4 ib = make_int4(trunc_i32(X1), trunc_i32(Y1), trunc_i32(X2), trunc_i32(Y2));
    const float4 fb = make_float4(X1, Y1, X2, Y2);
    const float sc = __uint_as_float(0xFFFFFFFFu - (uint32_t)(key >> 32));
    const int lab = p.mode == POST_FACE ? a : p.scratch_cls[(size_t)b * p.A + a];
    ((int4*)p.k_xyxy)[k] = ib;
    ((float4*)p.k_xyxy_f)[k] = fb;
    p.k_score[k] = sc;
    p.k_label[k] = lab;
    if (pos >= p.cap || !p.out_xyxy) return;
    const size_t o = (size_t)b * p.cap + pos;
    // caller arrays: scalar stores (no alignment assumed)
    p.out_xyxy[4 * o + 0] = ib.x; p.out_xyxy[4 * o + 1] = ib.y;
    p.out_xyxy[4 * o + 2] = ib.z; p.out_xyxy[4 * o + 3] = ib.w;
    if (p.out_xyxy_f) {
        p.out_xyxy_f[4 * o + 0] = X1; p.out_xyxy_f[4 * o + 1] = Y1;
        p.out_xyxy_f[4 * o + 2] = X2; p.out_xyxy_f[4 * o + 3] = Y2;
    }
    if (p.out_score) p.out_score[o] = sc;
    if (p.out_label) p.out_label[o] = lab;
}

__device__ void nms_frame(const PostArgs& p, int b, int M, uint64_t* keys, float4* box, float* area, uint8_t* supp,
                          uint64_t* chunk_keep, int* nkept_s) {
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    int P = 1;
    while (P < M) P <<= 1;
    const uint64_t* src = p.cand_keys + (size_t)b * p.A;
    for (int i = tid; i < P; i += NMS_THREADS) keys[i] = i < M ? src[i] : ~0ULL;
    __syncthreads();
    for (int k = 2; k <= P; k <<= 1) {            // bitonic sort, ascending
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = tid; i < P; i += NMS_THREADS) {
                const int ixj = i ^ j;
                if (ixj > i) {
                    const uint64_t ki = keys[i], kj = keys[ixj];
                    const bool up = (i & k) == 0;
                    if ((ki > kj) == up) { keys[i] = kj; keys[ixj] = ki; }
                }
            }
            __syncthreads();
        }
    }
    for (int i = tid; i < M; i += NMS_THREADS) {
        const int a = (int)(keys[i] & 0xFFFFFFFFu);
        float4 bx = p.scratch_box[(size_t)b * p.A + a];
        if (p.mode == POST_YOLO && p.max_wh != 0.f) {   // boxes + class * max_wh (class-aware NMS)
            const float off = VD_FMUL((float)p.scratch_cls[(size_t)b * p.A + a], p.max_wh);
            bx = make_float4(VD_FADD(bx.x, off), VD_FADD(bx.y, off), VD_FADD(bx.z, off), VD_FADD(bx.w, off));
        }
        box[i] = bx;
        area[i] = VD_FMUL(VD_FSUB(bx.z, bx.x), VD_FSUB(bx.w, bx.y));
        supp[i] = 0;
    }
    if (tid == 0) *nkept_s = 0;
    __syncthreads();

    const int limit = p.max_det > 0 ? min(p.max_det, p.kcap) : p.kcap;   // kcap >= every possible keep count
    for (int c0 = 0; c0 < M; c0 += 64) {
        if (wid == 0) {
            const int j = c0 + lane;
            const bool valid = j < M;
            const float4 bj = valid ? box[j] : make_float4(0, 0, 0, 0);
            const float aj = valid ? area[j] : 0.f;
            const bool alive = valid && !supp[j];
            uint64_t mask = 0;
            const int lim = min(64, M - c0);
            for (int k = lane + 1; k < lim; ++k) {
                const float4 bk = box[c0 + k];
                if (vd_iou_gt(bj.x, bj.y, bj.z, bj.w, aj, bk.x, bk.y, bk.z, bk.w, area[c0 + k], p.iou))
                    mask |= 1ULL << k;
            }
            uint64_t alive_bits = __ballot(alive);
            const uint32_t mlo = (uint32_t)mask, mhi = (uint32_t)(mask >> 32);
            for (int i = 0; i < lim; ++i) {
                if ((alive_bits >> i) & 1ULL) {
                    const uint64_t mi = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)mhi, i) << 32) |
                                        (uint32_t)__builtin_amdgcn_readlane((int)mlo, i);
                    alive_bits &= ~mi;
                }
            }
            const int base = *nkept_s;
            if ((alive_bits >> lane) & 1ULL) {
                const int pos = base + __popcll(alive_bits & ((1ULL << lane) - 1ULL));
                if (pos < limit) emit(p, b, pos, p.mode == POST_FACE ? bj : p.scratch_box[(size_t)b * p.A + (int)(keys[j] & 0xFFFFFFFFu)], keys[j]);
            }
            if (lane == 0) {
                *nkept_s = base + __popcll(alive_bits);
                *chunk_keep = alive_bits;
            }
        }
        __syncthreads();
        const uint64_t kb = *chunk_keep;
        if (kb) {
            for (int j = c0 + 64 + tid; j < M; j += NMS_THREADS) {
                if (supp[j]) continue;
                const float4 bj = box[j];
                const float aj = area[j];
                uint64_t bits = kb;
                while (bits) {
                    const int i = __ffsll((long long)bits) - 1;
                    bits &= bits - 1;
                    const float4 bi = box[c0 + i];
                    if (vd_iou_gt(bi.x, bi.y, bi.z, bi.w, area[c0 + i], bj.x, bj.y, bj.z, bj.w, aj, p.iou)) {
                        supp[j] = 1;
                        break;
                    }
                }
            }
        }
        __syncthreads();
    }
    if (tid == 0) {
        const int n = *nkept_s;
        const int kept = p.max_det > 0 ? min(n, p.max_det) : n;   // i = i[:max_det]
        p.k_count[b] = kept;
        if (p.out_count) p.out_count[b] = kept;
    }
}

__global__ __launch_bounds__(NMS_THREADS) void nms_kernel(PostArgs p) {
    __shared__ __attribute__((aligned(16))) float4 s_box[LDS_CAND];
    __shared__ __attribute__((aligned(16))) uint64_t s_keys[LDS_CAND];
    __shared__ float s_area[LDS_CAND];
    __shared__ uint8_t s_supp[LDS_CAND];
    __shared__ uint64_t s_chunk_keep;
    __shared__ int s_nkept;
    const int b = blockIdx.x;
    const int M = p.cand_count[b];
    if (M == 0) {
        if (threadIdx.x == 0) {
            p.k_count[b] = 0;
            if (p.out_count) p.out_count[b] = 0;
        }
        return;
    }
    if (M <= LDS_CAND)
        nms_frame(p, b, M, s_keys, s_box, s_area, s_supp, &s_chunk_keep, &s_nkept);
    else
        nms_frame(p, b, M, p.scratch_keys + (size_t)b * p.sort_cap, p.scratch_nbox + (size_t)b * p.A,
                  p.scratch_area + (size_t)b * p.A, p.scratch_supp + (size_t)b * p.A, &s_chunk_keep, &s_nkept);
}

}  // namespace

hipError_t vd_launch_post(const PostArgs& p, hipStream_t s) {
    hipError_t e = hipMemsetAsync(p.cand_count, 0, sizeof(int) * p.B, s);
    if (e != hipSuccess) return e;
    if (p.mode == POST_FACE)
        hipLaunchKernelGGL(face_candidates_kernel, dim3((p.A + 255) / 256, p.B), dim3(256), 0, s, p);
    else
        hipLaunchKernelGGL(yolo_candidates_kernel, dim3((p.A + 255) / 256, p.B), dim3(256), 0, s, p);
    hipLaunchKernelGGL(nms_kernel, dim3(p.B), dim3(NMS_THREADS), 0, s, p);
    return hipGetLastError();
}
