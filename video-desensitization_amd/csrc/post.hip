// post.hip — face post-processing on the GPU, bit-exact with the oracle.
//
// Replaces Retinaface.postprocess (detect_face/face.py:93-115) + the host
// scaling loop (face.py:136-148) + int() (combine_detect.py:243):
//   softmax score        retinaface.py:147           (vd_expf, float32 ops)
//   threshold >= conf    utils_bbox.py:115-116
//   decode               utils_bbox.py:49-59         (reference op order, no FMA)
//   batched_nms          utils_bbox.py:121-127 -> torchvision nms [ext]:
//                        stable descending sort, IoU in float32, '>' vs double
//   correct boxes        utils_bbox.py:12-43 (float32 tensors)
//   x [w,h,w,h]          face.py:144-145 (float32 numpy)
//   int()                combine_detect.py:243 (truncation toward zero)
//
// Two kernels per batch:
//  face_candidates_kernel: one thread per anchor, score + threshold, survivors
//    compacted into a per-frame key list (64-bit key = (~score_bits, anchor) so
//    an ascending sort is the stable descending-score order torchvision uses).
//  face_nms_kernel: one 1024-thread workgroup per frame. Bitonic sort of the
//    keys, decode of the survivors, then greedy NMS in chunks of 64: wave 0
//    resolves a chunk with a 64x64 IoU bitmask and a scalar sweep
//    (readlane), then all 16 waves suppress the later candidates against the
//    chunk's kept boxes. Result = exactly the sequential greedy keep list.
//    Small candidate sets live in LDS, large ones in a global scratch.
#include "vd_common.h"
#include "vd_math.h"

namespace {

constexpr int NMS_THREADS = 1024;
constexpr int LDS_CAND = 2048;     // candidates held in LDS; more -> global scratch

__global__ __launch_bounds__(256) void face_candidates_kernel(FacePostArgs p) {
    const int a = blockIdx.x * 256 + threadIdx.x;
    const int b = blockIdx.y;
    if (a >= p.A) return;
    int l = a >= p.loff[2] ? 2 : (a >= p.loff[1] ? 1 : 0);
    int local = a - p.loff[l];
    int pix = local >> 1, k = local & 1;
    const float* h = p.heads[l] + ((size_t)b * p.lh[l] * p.lw[l] + pix) * 32;
    float c0 = h[8 + 2 * k], c1 = h[9 + 2 * k];
    float m = c0 > c1 ? c0 : c1;
    float e0 = vd_expf(VD_FSUB(c0, m));
    float e1 = vd_expf(VD_FSUB(c1, m));
    float s = VD_FDIV(e1, VD_FADD(e0, e1));
    if (s >= p.conf) {
        int pos = atomicAdd(&p.cand_count[b], 1);
        uint32_t bits = __float_as_uint(s);
        p.cand_keys[(size_t)b * p.A + pos] = ((uint64_t)(0xFFFFFFFFu - bits) << 32) | (uint32_t)a;
    }
}

__device__ __forceinline__ float4 decode_box(const FacePostArgs& p, int b, int a) {
    int l = a >= p.loff[2] ? 2 : (a >= p.loff[1] ? 1 : 0);
    int local = a - p.loff[l];
    int pix = local >> 1, k = local & 1;
    const float* h = p.heads[l] + ((size_t)b * p.lh[l] * p.lw[l] + pix) * 32 + 4 * k;
    const float4 pr = *(const float4*)(p.anchors + 4 * (size_t)a);
    const float v0 = 0.1f, v1 = 0.2f;
    float cx = VD_FADD(pr.x, VD_FMUL(VD_FMUL(h[0], v0), pr.z));
    float cy = VD_FADD(pr.y, VD_FMUL(VD_FMUL(h[1], v0), pr.w));
    float w = VD_FMUL(pr.z, vd_expf(VD_FMUL(h[2], v1)));
    float hh = VD_FMUL(pr.w, vd_expf(VD_FMUL(h[3], v1)));
    float x1 = VD_FSUB(cx, VD_FDIV(w, 2.0f));
    float y1 = VD_FSUB(cy, VD_FDIV(hh, 2.0f));
    return make_float4(x1, y1, VD_FADD(w, x1), VD_FADD(hh, y1));
}

__device__ __forceinline__ int trunc_i32(float v) {
    // int(x) of a Python float; values beyond int32 are clamped (the mosaic clips
    // to the frame first, combine_detect.py:145-148, so the output is unchanged).
    if (!(v == v)) return 0;
    if (v >= 2147483520.0f) return 2147483647;
    if (v <= -2147483648.0f) return (-2147483647 - 1);
    return (int)v;   // truncation toward zero
}

template <bool IN_LDS>
__device__ void nms_frame(const FacePostArgs& p, int b, int M, uint64_t* keys, float4* box, float* area,
                          uint8_t* supp, uint64_t* chunk_keep, int* nkept_s) {
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    int P = 1;
    while (P < M) P <<= 1;
    const uint64_t* src = p.cand_keys + (size_t)b * p.A;
    for (int i = tid; i < P; i += NMS_THREADS) keys[i] = i < M ? src[i] : ~0ULL;
    __syncthreads();
    // bitonic sort, ascending
    for (int k = 2; k <= P; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = tid; i < P; i += NMS_THREADS) {
                int ixj = i ^ j;
                if (ixj > i) {
                    uint64_t ki = keys[i], kj = keys[ixj];
                    bool up = (i & k) == 0;
                    if ((ki > kj) == up) { keys[i] = kj; keys[ixj] = ki; }
                }
            }
            __syncthreads();
        }
    }
    for (int i = tid; i < M; i += NMS_THREADS) {
        float4 bx = decode_box(p, b, (int)(keys[i] & 0xFFFFFFFFu));
        box[i] = bx;
        area[i] = VD_FMUL(VD_FSUB(bx.z, bx.x), VD_FSUB(bx.w, bx.y));
        supp[i] = 0;
    }
    if (tid == 0) *nkept_s = 0;
    __syncthreads();

    // source -> output geometry (utils_bbox.py:118-132, float32)
    const float inh = (float)p.in_h, inw = (float)p.in_w, ih = (float)p.img_h, iw = (float)p.img_w;
    const float rh = VD_FDIV(inh, ih), rw = VD_FDIV(inw, iw);
    const float mn = rh < rw ? rh : rw;
    const float nh = VD_FMUL(ih, mn), nw = VD_FMUL(iw, mn);
    const float offy = VD_FDIV(VD_FDIV(VD_FSUB(inh, nh), 2.0f), inh);
    const float offx = VD_FDIV(VD_FDIV(VD_FSUB(inw, nw), 2.0f), inw);
    const float scy = VD_FDIV(inh, nh), scx = VD_FDIV(inw, nw);

    for (int c0 = 0; c0 < M; c0 += 64) {
        if (wid == 0) {
            const int j = c0 + lane;
            const bool valid = j < M;
            float4 bj = valid ? box[j] : make_float4(0, 0, 0, 0);
            float aj = valid ? area[j] : 0.f;
            bool alive = valid && !supp[j];
            uint64_t mask = 0;
            const int lim = min(64, M - c0);
            for (int k = lane + 1; k < lim; ++k) {
                float4 bk = box[c0 + k];
                if (vd_iou_gt(bj.x, bj.y, bj.z, bj.w, aj, bk.x, bk.y, bk.z, bk.w, area[c0 + k], p.iou))
                    mask |= 1ULL << k;
            }
            uint64_t alive_bits = __ballot(alive);
            const uint32_t mlo = (uint32_t)mask, mhi = (uint32_t)(mask >> 32);
            for (int i = 0; i < lim; ++i) {
                if ((alive_bits >> i) & 1ULL) {
                    uint64_t mi = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)mhi, i) << 32) |
                                  (uint32_t)__builtin_amdgcn_readlane((int)mlo, i);
                    alive_bits &= ~mi;
                }
            }
            const int base = *nkept_s;
            const bool keep = (alive_bits >> lane) & 1ULL;
            if (keep) {
                const int pos = base + __popcll(alive_bits & ((1ULL << lane) - 1ULL));
                if (pos < p.cap) {
                    const size_t o = (size_t)b * p.cap + pos;
                    // (box - offset) * scale, then * [w, h, w, h]
                    float X1 = VD_FMUL(VD_FMUL(VD_FSUB(bj.x, offx), scx), iw);
                    float Y1 = VD_FMUL(VD_FMUL(VD_FSUB(bj.y, offy), scy), ih);
                    float X2 = VD_FMUL(VD_FMUL(VD_FSUB(bj.z, offx), scx), iw);
                    float Y2 = VD_FMUL(VD_FMUL(VD_FSUB(bj.w, offy), scy), ih);
                    p.out_xyxy[4 * o + 0] = trunc_i32(X1);
                    p.out_xyxy[4 * o + 1] = trunc_i32(Y1);
                    p.out_xyxy[4 * o + 2] = trunc_i32(X2);
                    p.out_xyxy[4 * o + 3] = trunc_i32(Y2);
                    if (p.out_xyxy_f) {
                        p.out_xyxy_f[4 * o + 0] = X1; p.out_xyxy_f[4 * o + 1] = Y1;
                        p.out_xyxy_f[4 * o + 2] = X2; p.out_xyxy_f[4 * o + 3] = Y2;
                    }
                    const uint64_t key = keys[j];
                    if (p.out_score) p.out_score[o] = __uint_as_float(0xFFFFFFFFu - (uint32_t)(key >> 32));
                    if (p.out_label) p.out_label[o] = (int)(key & 0xFFFFFFFFu);
                }
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
    if (tid == 0) p.out_count[b] = *nkept_s;
}

__global__ __launch_bounds__(NMS_THREADS) void face_nms_kernel(FacePostArgs p) {
    __shared__ __attribute__((aligned(16))) float4 s_box[LDS_CAND];
    __shared__ __attribute__((aligned(16))) uint64_t s_keys[LDS_CAND];
    __shared__ float s_area[LDS_CAND];
    __shared__ uint8_t s_supp[LDS_CAND];
    __shared__ uint64_t s_chunk_keep;
    __shared__ int s_nkept;
    const int b = blockIdx.x;
    const int M = p.cand_count[b];
    if (M == 0) {
        if (threadIdx.x == 0) p.out_count[b] = 0;
        return;
    }
    if (M <= LDS_CAND) {
        nms_frame<true>(p, b, M, s_keys, s_box, s_area, s_supp, &s_chunk_keep, &s_nkept);
    } else {
        nms_frame<false>(p, b, M, p.scratch_keys + (size_t)b * p.sort_cap, p.scratch_box + (size_t)b * p.A,
                         p.scratch_area + (size_t)b * p.A, p.scratch_supp + (size_t)b * p.A,
                         &s_chunk_keep, &s_nkept);
    }
}

}  // namespace

hipError_t vd_launch_face_post(const FacePostArgs& p, hipStream_t s) {
    hipError_t e = hipMemsetAsync(p.cand_count, 0, sizeof(int) * p.B, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(face_candidates_kernel, dim3((p.A + 255) / 256, p.B), dim3(256), 0, s, p);
    hipLaunchKernelGGL(face_nms_kernel, dim3(p.B), dim3(NMS_THREADS), 0, s, p);
    return hipGetLastError();
}
