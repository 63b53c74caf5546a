// mosaic.hip — out-of-place pixelation of detected boxes, exact reference semantics.
//
// Replaces combine_detect.py:246-249 (img.copy() + per box, in order,
// mosaic_rectangle_region_single :138-161: clip, cv2.resize INTER_NEAREST down
// to (max(1,bw//L), max(1,bh//L)) and back up [ext resizeNN], write back).
// Box k reads the output of box k-1, so a pixel's value is found by walking the
// box list BACKWARDS: p <- map_k(p) for every box k (last to first) that
// contains p, then out(p) = in(p'). map_k = down(up(.)) per axis with OpenCV's
// double-precision nearest index rule. This is a pure gather -> |delta| = 0.
//
// Kernels per call:
//  mosaic_prep_kernel  one thread per box: clip to the frame and precompute the
//                      four resizeNN factors into a per-frame table (boxes in
//                      call order: faces first, then plates, combine_detect.py:242-244).
//  mosaic_copy_kernel  the img.copy() of :247 — a 64-B-per-thread streaming copy
//                      of every frame with <= BOX_FAST boxes (HBM roofline).
//  mosaic_box_kernel   one workgroup slice per (frame, box k): for each pixel of
//                      box k that no LATER box contains (that box owns it), walk
//                      k, k-1, ..., 0 and gather the 3 source bytes. Only covered
//                      pixels are touched; the frame's box table sits in LDS.
//  mosaic_kernel       fallback for frames with > BOX_FAST boxes: one workgroup
//                      per (frame, band of ROWS rows). The band's box list (table
//                      entries intersecting the band, original order) is staged
//                      in LDS; a 16-byte chunk no band box touches is a vector
//                      copy, the rest walk per pixel. A walk that leaves the band
//                      (points only move up/left) continues on the frame's full
//                      table, so the band list is an exact filter.
// HBM traffic = read + write of every frame (2*W*H*3 bytes) + ROI gathers (L2 hits).
#include "vd_common.h"
#include "vd_math.h"

#include <algorithm>

namespace {

constexpr int ROWS = 8;
constexpr int TB_CAP = 512;    // band-list capacity; larger bands walk the global table
constexpr int BOX_FAST = 256;  // frames with at most this many boxes take copy + box kernels
constexpr int BOX_BLOCKS = 256; // workgroups per frame sharing its box pixels

struct MBox { int x1, y1, x2, y2; int sw, sh, idx, valid; double fux, fdx, fuy, fdy; };

struct MosaicArgs {
    const uint8_t* in; uint8_t* out; int n, h, w; size_t pitch;
    const int* cnt0; const int* xy0; int cap0;      // list 0 (faces)
    const int* cnt1; const int* xy1; int cap1;      // list 1 (plates, optional)
    int level;
    int vec_ok;                                      // 16-B aligned rows -> vector copies
    MBox* table; int tcap;                           // [n][tcap] prepared boxes
    uint64_t* ovl;                                   // [n][BOX_FAST][4] overlap bitmasks (fast path)
    int* pref;                                       // [n][BOX_FAST+1] prefix sums of box areas (fast path)
};

__global__ __launch_bounds__(256) void mosaic_prep_kernel(MosaicArgs a) {
    const int k = blockIdx.x * 256 + threadIdx.x;
    const int f = blockIdx.y;
    if (k >= a.tcap) return;
    const int n0 = a.cnt0 ? min(a.cnt0[f], a.cap0) : 0;
    const int n1 = a.cnt1 ? min(a.cnt1[f], a.cap1) : 0;
    if (k >= n0 + n1) return;
    const int* src = k < n0 ? a.xy0 + ((size_t)f * a.cap0 + k) * 4 : a.xy1 + ((size_t)f * a.cap1 + (k - n0)) * 4;
    MBox m{};
    // combine_detect.py:145-148 clip, :150-151 empty check
    m.x1 = max(0, src[0]); m.y1 = max(0, src[1]);
    m.x2 = min(a.w, src[2]); m.y2 = min(a.h, src[3]);
    m.idx = k;
    m.valid = (m.x2 > m.x1 && m.y2 > m.y1) ? 1 : 0;
    if (m.valid) {
        const int bw = m.x2 - m.x1, bh = m.y2 - m.y1;
        m.sw = max(1, bw / a.level);              // :153-154
        m.sh = max(1, bh / a.level);
        // resizeNN [ext]: ifx = 1. / ((double)dst / src)
        m.fux = __ddiv_rn(1.0, __ddiv_rn((double)bw, (double)m.sw));   // up:   dst=bw, src=sw
        m.fdx = __ddiv_rn(1.0, __ddiv_rn((double)m.sw, (double)bw));   // down: dst=sw, src=bw
        m.fuy = __ddiv_rn(1.0, __ddiv_rn((double)bh, (double)m.sh));
        m.fdy = __ddiv_rn(1.0, __ddiv_rn((double)m.sh, (double)bh));
    }
    a.table[(size_t)f * a.tcap + k] = m;
}

__device__ __forceinline__ void apply(const MBox& m, int& y, int& x) {
    int ux = min((int)floor(VD_DMUL((double)(x - m.x1), m.fux)), m.sw - 1);
    int dx = min((int)floor(VD_DMUL((double)ux, m.fdx)), m.x2 - m.x1 - 1);
    int uy = min((int)floor(VD_DMUL((double)(y - m.y1), m.fuy)), m.sh - 1);
    int dy = min((int)floor(VD_DMUL((double)uy, m.fdy)), m.y2 - m.y1 - 1);
    x = m.x1 + dx;
    y = m.y1 + dy;
}

__device__ __forceinline__ bool inside(const MBox& m, int y, int x) {
    return x >= m.x1 && x < m.x2 && y >= m.y1 && y < m.y2;
}

__global__ __launch_bounds__(256) void mosaic_kernel(MosaicArgs a) {
    __shared__ MBox s_box[TB_CAP];
    __shared__ int s_n;
    __shared__ int s_wsum[4];
    const int f = blockIdx.y;
    const int y0 = blockIdx.x * ROWS;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int n0 = a.cnt0 ? min(a.cnt0[f], a.cap0) : 0;
    const int n1 = a.cnt1 ? min(a.cnt1[f], a.cap1) : 0;
    const int nb = n0 + n1;
    if (nb <= BOX_FAST) return;        // copy + box kernels own this frame
    const MBox* table = a.table + (size_t)f * a.tcap;
    if (tid == 0) s_n = 0;
    __syncthreads();
    // ordered compaction of the boxes intersecting rows [y0, y0+ROWS)
    for (int base = 0; base < nb; base += 256) {
        const int k = base + tid;
        MBox m;
        bool hit = false;
        if (k < nb) {
            m = table[k];
            hit = m.valid && m.y1 < y0 + ROWS && m.y2 > y0;
        }
        const uint64_t bal = __ballot(hit);
        const int wpre = __popcll(bal & ((1ULL << lane) - 1ULL));
        if (lane == 0) s_wsum[wid] = __popcll(bal);
        __syncthreads();
        int off = s_n;
        for (int i = 0; i < wid; ++i) off += s_wsum[i];
        if (hit && off + wpre < TB_CAP) s_box[off + wpre] = m;
        __syncthreads();
        if (tid == 0) s_n += s_wsum[0] + s_wsum[1] + s_wsum[2] + s_wsum[3];
        __syncthreads();
    }
    const bool overflow = s_n > TB_CAP;
    const int nt = min(s_n, TB_CAP);

    const uint8_t* src = a.in + (size_t)f * a.h * a.pitch;
    uint8_t* dst = a.out + (size_t)f * a.h * a.pitch;
    const int row_bytes = a.w * 3;
    const int nchunk = (row_bytes + 15) >> 4;

    auto walk = [&](int y, int x, int& sy, int& sx) {
        int next_global = nb - 1;       // table index still to consider
        bool in_band = !overflow;
        if (in_band) {
            for (int t = nt - 1; t >= 0; --t) {
                const MBox& m = s_box[t];
                if (inside(m, y, x)) {
                    apply(m, y, x);
                    if (y < y0) { next_global = m.idx - 1; in_band = false; break; }
                }
            }
        }
        if (!in_band) {
            for (int k = next_global; k >= 0; --k) {
                const MBox m = table[k];
                if (m.valid && inside(m, y, x)) apply(m, y, x);
            }
        }
        sy = y; sx = x;
    };

    for (int r = 0; r < ROWS; ++r) {
        const int y = y0 + r;
        if (y >= a.h) break;
        const uint8_t* srow = src + (size_t)y * a.pitch;
        uint8_t* drow = dst + (size_t)y * a.pitch;
        for (int c = tid; c < nchunk; c += 256) {
            const int b0 = c << 4;
            const int bend = min(b0 + 16, row_bytes);
            const int px0 = b0 / 3, px1 = (bend - 1) / 3;
            bool touched = overflow;
            for (int t = 0; t < nt && !touched; ++t) {
                const MBox& m = s_box[t];
                touched = y >= m.y1 && y < m.y2 && px1 >= m.x1 && px0 < m.x2;
            }
            if (!touched && bend - b0 == 16 && a.vec_ok) {
                *(uint4*)(drow + b0) = *(const uint4*)(srow + b0);
                continue;
            }
            uint8_t tmp[16];
            int lastx = -1, sy = 0, sx = 0;
            for (int bb = b0; bb < bend; ++bb) {
                const int x = bb / 3, ch = bb - 3 * x;
                if (x != lastx) {
                    if (touched) walk(y, x, sy, sx); else { sy = y; sx = x; }
                    lastx = x;
                }
                tmp[bb - b0] = src[(size_t)sy * a.pitch + sx * 3 + ch];
            }
            if (bend - b0 == 16 && a.vec_ok) *(uint4*)(drow + b0) = *(const uint4*)tmp;
            else for (int bb = b0; bb < bend; ++bb) drow[bb] = tmp[bb - b0];
        }
    }
}

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// img.copy() for the frames of the fast path: 4 x 16 B per thread per iteration.
__global__ __launch_bounds__(256) void mosaic_copy_kernel(MosaicArgs a) {
    const int f = blockIdx.y;
    const int n0 = a.cnt0 ? min(a.cnt0[f], a.cap0) : 0;
    const int n1 = a.cnt1 ? min(a.cnt1[f], a.cap1) : 0;
    if (n0 + n1 > BOX_FAST) return;
    const size_t bytes = (size_t)a.h * a.pitch;
    const uint8_t* src = a.in + (size_t)f * bytes;
    uint8_t* dst = a.out + (size_t)f * bytes;
    if (a.vec_ok) {
        const size_t nv = bytes >> 4;
        const u32x4* s4 = (const u32x4*)src;
        u32x4* d4 = (u32x4*)dst;
        const size_t stride = (size_t)gridDim.x * 256;
        size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
        for (; i + 3 * stride < nv; i += 4 * stride) {
            const u32x4 v0 = s4[i], v1 = s4[i + stride], v2 = s4[i + 2 * stride], v3 = s4[i + 3 * stride];
            d4[i] = v0; d4[i + stride] = v1; d4[i + 2 * stride] = v2; d4[i + 3 * stride] = v3;
        }
        for (; i < nv; i += stride) d4[i] = s4[i];
        for (size_t t = (nv << 4) + (size_t)blockIdx.x * 256 + threadIdx.x; t < bytes; t += stride) dst[t] = src[t];
    } else {
        for (size_t t = (size_t)blockIdx.x * 256 + threadIdx.x; t < bytes; t += (size_t)gridDim.x * 256) dst[t] = src[t];
    }
}

// Overlap graph of the fast-path frames: bit j of ovl[k] <=> boxes j and k intersect.
__global__ __launch_bounds__(256) void mosaic_overlap_kernel(MosaicArgs a) {
    const int f = blockIdx.y;
    const int k = threadIdx.x;
    const int n0 = a.cnt0 ? min(a.cnt0[f], a.cap0) : 0;
    const int n1 = a.cnt1 ? min(a.cnt1[f], a.cap1) : 0;
    const int nb = n0 + n1;
    if (nb > BOX_FAST || k >= nb) return;
    const MBox* t = a.table + (size_t)f * a.tcap;
    uint64_t m[4] = {0, 0, 0, 0};
    const MBox bk = t[k];
    if (bk.valid)
        for (int j = 0; j < nb; ++j) {
            const MBox bj = t[j];
            if (j != k && bj.valid && bj.x1 < bk.x2 && bk.x1 < bj.x2 && bj.y1 < bk.y2 && bk.y1 < bj.y2)
                m[j >> 6] |= 1ULL << (j & 63);
        }
    uint64_t* o = a.ovl + ((size_t)f * BOX_FAST + k) * 4;
    o[0] = m[0]; o[1] = m[1]; o[2] = m[2]; o[3] = m[3];
}

// Per frame: exclusive prefix sum of the valid boxes' pixel counts (one block per frame).
__global__ __launch_bounds__(256) void mosaic_prefix_kernel(MosaicArgs a) {
    __shared__ int s[256];
    const int f = blockIdx.x, k = threadIdx.x;
    const int n0 = a.cnt0 ? min(a.cnt0[f], a.cap0) : 0;
    const int n1 = a.cnt1 ? min(a.cnt1[f], a.cap1) : 0;
    const int nb = n0 + n1;
    int* pref = a.pref + (size_t)f * (BOX_FAST + 1);
    if (nb > BOX_FAST) { if (k == 0) pref[0] = 0; return; }
    int v = 0;
    if (k < nb) {
        const MBox b = a.table[(size_t)f * a.tcap + k];
        if (b.valid) v = (b.x2 - b.x1) * (b.y2 - b.y1);
    }
    s[k] = v;
    __syncthreads();
    for (int off = 1; off < 256; off <<= 1) {      // Hillis-Steele inclusive scan
        const int t = k >= off ? s[k - off] : 0;
        __syncthreads();
        s[k] += t;
        __syncthreads();
    }
    if (k <= nb) pref[k] = k == 0 ? 0 : s[k - 1];
}

// Highest set bit index < lim in a 256-bit mask, or -1.
__device__ __forceinline__ int top_below(const uint64_t* m, int lim) {
    for (int w = (lim - 1) >> 6; w >= 0; --w) {
        uint64_t v = m[w];
        const int hi = lim - (w << 6);               // bits [0, hi) of this word are eligible
        if (hi < 64) v &= (1ULL << hi) - 1ULL;
        if (v) return (w << 6) + 63 - __clzll((long long)v);
    }
    return -1;
}

// Pixels of box k that no LATER box contains: walk k, then earlier boxes along the
// overlap graph (a box containing a point of box j overlaps j), gather 3 bytes.
// Work is balanced over the frame's flattened box-pixel index space
// [0, sum of box areas): workgroup g of BOX_BLOCKS takes a strided share, and a
// binary search over the area prefix sums maps an index to (box, pixel).
__global__ __launch_bounds__(256) void mosaic_box_kernel(MosaicArgs a) {
    __shared__ MBox s_tab[BOX_FAST];
    __shared__ uint64_t s_ovl[BOX_FAST][4];
    __shared__ int s_pref[BOX_FAST + 1];
    const int f = blockIdx.y;
    const int n0 = a.cnt0 ? min(a.cnt0[f], a.cap0) : 0;
    const int n1 = a.cnt1 ? min(a.cnt1[f], a.cap1) : 0;
    const int nb = n0 + n1;
    if (nb > BOX_FAST || nb == 0) return;
    const int* pref = a.pref + (size_t)f * (BOX_FAST + 1);
    const int total = pref[nb];
    if (blockIdx.x * 256 >= total) return;
    const MBox* table = a.table + (size_t)f * a.tcap;
    const uint64_t* ovl = a.ovl + (size_t)f * BOX_FAST * 4;
    for (int i = threadIdx.x; i < nb; i += 256) {
        s_tab[i] = table[i];
        s_ovl[i][0] = ovl[4 * i + 0]; s_ovl[i][1] = ovl[4 * i + 1];
        s_ovl[i][2] = ovl[4 * i + 2]; s_ovl[i][3] = ovl[4 * i + 3];
    }
    for (int i = threadIdx.x; i <= nb; i += 256) s_pref[i] = pref[i];
    __syncthreads();
    const uint8_t* src = a.in + (size_t)f * a.h * a.pitch;
    uint8_t* dst = a.out + (size_t)f * a.h * a.pitch;
    for (int t = blockIdx.x * 256 + threadIdx.x; t < total; t += gridDim.x * 256) {
        int lo = 0, hi = nb - 1;                    // largest k with s_pref[k] <= t
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (s_pref[mid] <= t) lo = mid; else hi = mid - 1;
        }
        const int k = lo;
        const MBox& bk = s_tab[k];
        const int bw = bk.x2 - bk.x1;
        const int p = t - s_pref[k];
        const int py = p / bw;
        const int y0 = bk.y1 + py, x0 = bk.x1 + (p - py * bw);
        bool owned = true;
        for (int w = (k + 1) >> 6; w < 4 && owned; ++w) {       // later boxes overlapping k
            uint64_t v = s_ovl[k][w];
            const int lo_bit = k + 1 - (w << 6);
            if (lo_bit > 0) v &= ~((1ULL << lo_bit) - 1ULL);
            while (v && owned) {
                const int j = (w << 6) + __ffsll((long long)v) - 1;
                v &= v - 1;
                owned = !inside(s_tab[j], y0, x0);
            }
        }
        if (!owned) continue;
        int y = y0, x = x0;
        apply(bk, y, x);
        int cur = k;
        for (;;) {   // next (highest-index, earlier) box containing the point, along the overlap graph
            int lim = cur, j;
            while ((j = top_below(s_ovl[cur], lim)) >= 0 && !inside(s_tab[j], y, x)) lim = j;
            if (j < 0) break;
            apply(s_tab[j], y, x);
            cur = j;
        }
        const uint8_t* sp = src + (size_t)y * a.pitch + x * 3;
        uint8_t* dp = dst + (size_t)y0 * a.pitch + x0 * 3;
        const uint8_t c0 = sp[0], c1 = sp[1], c2 = sp[2];
        dp[0] = c0; dp[1] = c1; dp[2] = c2;
    }
}

}  // namespace

size_t vd_mosaic_table_bytes(int n, int tcap) {
    return (size_t)n * tcap * sizeof(MBox) + (size_t)n * BOX_FAST * 32 + (size_t)n * (BOX_FAST + 1) * 4;
}

hipError_t vd_launch_mosaic(const uint8_t* in, uint8_t* out, int n, int h, int w, size_t pitch,
                            const int* cnt0, const int* xy0, int cap0,
                            const int* cnt1, const int* xy1, int cap1, int level, void* table,
                            hipStream_t s) {
    const int vec_ok = (pitch % 16 == 0) && ((uintptr_t)in % 16 == 0) && ((uintptr_t)out % 16 == 0);
    const int tcap = (cnt0 ? cap0 : 0) + (cnt1 ? cap1 : 0);
    char* tail = (char*)table + (size_t)n * tcap * sizeof(MBox);
    MosaicArgs a{in, out, n, h, w, pitch, cnt0, xy0, cap0, cnt1, xy1, cap1, level, vec_ok, (MBox*)table, tcap,
                 (uint64_t*)tail, (int*)(tail + (size_t)n * BOX_FAST * 32)};
    if (tcap > 0)
        hipLaunchKernelGGL(mosaic_prep_kernel, dim3((tcap + 255) / 256, n), dim3(256), 0, s, a);
    // fast path: copy (~1 MiB per workgroup row of the grid) then owned-pixel gathers
    const size_t fbytes = (size_t)h * pitch;
    const int cblocks = (int)std::min<size_t>(1024, std::max<size_t>(1, fbytes / (64 * 256 * 4)));
    hipLaunchKernelGGL(mosaic_copy_kernel, dim3(cblocks, n), dim3(256), 0, s, a);
    if (tcap > 0) {
        hipLaunchKernelGGL(mosaic_overlap_kernel, dim3(1, n), dim3(256), 0, s, a);
        hipLaunchKernelGGL(mosaic_prefix_kernel, dim3(n), dim3(256), 0, s, a);
        hipLaunchKernelGGL(mosaic_box_kernel, dim3(BOX_BLOCKS, n), dim3(256), 0, s, a);
        // frames with more boxes than the fast path holds
        hipLaunchKernelGGL(mosaic_kernel, dim3((h + ROWS - 1) / ROWS, n), dim3(256), 0, s, a);
    }
    return hipGetLastError();
}
