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
//  mosaic_prefix_kernel per frame: prefix sums of the boxes' pixel counts and of
//                      their mosaic cell counts (sw*sh), for balanced flat grids.
//  mosaic_cell_kernel  one thread per mosaic CELL (ux, uy) of every box: all the
//                      pixels of a cell map to the same point, so the backward
//                      walk over earlier boxes and the 3-byte gather run once per
//                      cell (level^2 fewer times than per pixel) into a cell table.
//  mosaic_box_kernel   every pixel of box k that no LATER box contains (box k owns
//                      it) takes its cell's colour. Work is flat over the frame's
//                      box pixels; the frame's box table sits in LDS. (Frames whose
//                      cells exceed the table walk per pixel instead.)
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
constexpr int CELL_BLOCKS = 32; // workgroups per frame sharing its mosaic cells
constexpr int CELL_CAP = 1 << 18;   // cell-table entries per frame (packed RGB)

struct MBox { int x1, y1, x2, y2; int sw, sh, idx, valid; double fux, fdx, fuy, fdy; };

struct MosaicArgs {
    const uint8_t* in; uint8_t* out; int n, h, w; size_t pitch;
    const int* cnt0; const int* xy0; int cap0;      // list 0 (faces)
    const int* cnt1; const int* xy1; int cap1;      // list 1 (plates, optional)
    int level;
    int vec_ok;                                      // 16-B aligned rows -> vector copies
    MBox* table; int tcap;                           // [n][tcap] prepared boxes
    uint64_t* ovl;                                   // [n][BOX_FAST][4] overlap bitmasks (fast path)
    int* pref;                                       // [n][BOX_FAST+1] prefix sums of box quads (fast path)
    int* cpref;                                      // [n][BOX_FAST+1] prefix sums of box cells sw*sh
    uint32_t* cells;                                 // [n][CELL_CAP] walked colour per cell
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
    int* cpref = a.cpref + (size_t)f * (BOX_FAST + 1);
    if (nb > BOX_FAST) { if (k == 0) { pref[0] = 0; cpref[0] = 0; } return; }
    MBox b{};
    if (k < nb) b = a.table[(size_t)f * a.tcap + k];
    for (int pass = 0; pass < 2; ++pass) {
        int v = 0;
        // pass 0: 4-pixel quads (aligned to absolute x % 4) per box; pass 1: mosaic cells
        if (k < nb && b.valid) v = pass == 0 ? (((b.x2 - 1) >> 2) - (b.x1 >> 2) + 1) * (b.y2 - b.y1) : b.sw * b.sh;
        s[k] = v;
        __syncthreads();
        for (int off = 1; off < 256; off <<= 1) {      // Hillis-Steele inclusive scan
            const int t = k >= off ? s[k - off] : 0;
            __syncthreads();
            s[k] += t;
            __syncthreads();
        }
        if (k <= nb) (pass == 0 ? pref : cpref)[k] = k == 0 ? 0 : s[k - 1];
        __syncthreads();
    }
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

__device__ __forceinline__ int find_box(const int* pref, int nb, int t) {   // largest k with pref[k] <= t
    int lo = 0, hi = nb - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (pref[mid] <= t) lo = mid; else hi = mid - 1;
    }
    return lo;
}

// Walk a point already mapped by box `cur` back through the earlier boxes that
// contain it (the highest-index earlier box first, along the overlap graph).
__device__ __forceinline__ void walk_back(const MBox* tab, const uint64_t (*ovl)[4], int cur, int& y, int& x) {
    for (;;) {
        int lim = cur, j;
        while ((j = top_below(ovl[cur], lim)) >= 0 && !inside(tab[j], y, x)) lim = j;
        if (j < 0) break;
        apply(tab[j], y, x);
        cur = j;
    }
}

// One thread per mosaic cell of every box of a fast-path frame (flat over the
// frame's cells): map, walk, gather the colour into the cell table.
__global__ __launch_bounds__(256) void mosaic_cell_kernel(MosaicArgs a) {
    __shared__ MBox s_tab[BOX_FAST];
    __shared__ uint64_t s_ovl[BOX_FAST][4];
    __shared__ int s_cpref[BOX_FAST + 1];
    const int f = blockIdx.y;
    const int n0 = a.cnt0 ? min(a.cnt0[f], a.cap0) : 0;
    const int n1 = a.cnt1 ? min(a.cnt1[f], a.cap1) : 0;
    const int nb = n0 + n1;
    if (nb > BOX_FAST || nb == 0) return;
    const int* cpref = a.cpref + (size_t)f * (BOX_FAST + 1);
    const int total = cpref[nb];
    if (total > CELL_CAP || blockIdx.x * 256 >= total) return;
    const MBox* table = a.table + (size_t)f * a.tcap;
    const uint64_t* ovl = a.ovl + (size_t)f * BOX_FAST * 4;
    for (int i = threadIdx.x; i < nb; i += 256) {
        s_tab[i] = table[i];
        s_ovl[i][0] = ovl[4 * i + 0]; s_ovl[i][1] = ovl[4 * i + 1];
        s_ovl[i][2] = ovl[4 * i + 2]; s_ovl[i][3] = ovl[4 * i + 3];
    }
    for (int i = threadIdx.x; i <= nb; i += 256) s_cpref[i] = cpref[i];
    __syncthreads();
    const uint8_t* src = a.in + (size_t)f * a.h * a.pitch;
    uint32_t* cells = a.cells + (size_t)f * CELL_CAP;
    for (int t = blockIdx.x * 256 + threadIdx.x; t < total; t += gridDim.x * 256) {
        const int k = find_box(s_cpref, nb, t);
        const MBox& bk = s_tab[k];
        const int c = t - s_cpref[k];
        const int uy = c / bk.sw, ux = c - uy * bk.sw;
        // apply(bk) of any pixel of this cell: the down-mapped point of (ux, uy)
        int x = bk.x1 + min((int)floor(VD_DMUL((double)ux, bk.fdx)), bk.x2 - bk.x1 - 1);
        int y = bk.y1 + min((int)floor(VD_DMUL((double)uy, bk.fdy)), bk.y2 - bk.y1 - 1);
        walk_back(s_tab, s_ovl, k, y, x);
        const uint8_t* sp = src + (size_t)y * a.pitch + x * 3;
        cells[t] = (uint32_t)sp[0] | ((uint32_t)sp[1] << 8) | ((uint32_t)sp[2] << 16);
    }
}

// Pixels of box k that no LATER box contains take the colour of their cell
// (or, when the frame's cells overflow the table, walk per pixel).
// Work is balanced over the frame's flattened index space of box QUADS (4
// pixels x .. x+3 of one row, x % 4 == 0, clipped to the box): workgroup g of
// BOX_BLOCKS takes a strided share, and a binary search over the quad prefix sums
// maps an index to (box, row, quad). A fully owned quad is one 12-B store.
__global__ __launch_bounds__(256) void mosaic_box_kernel(MosaicArgs a) {
    __shared__ MBox s_tab[BOX_FAST];
    __shared__ uint64_t s_ovl[BOX_FAST][4];
    __shared__ int s_pref[BOX_FAST + 1];
    __shared__ int s_cpref[BOX_FAST + 1];
    const int f = blockIdx.y;
    const int n0 = a.cnt0 ? min(a.cnt0[f], a.cap0) : 0;
    const int n1 = a.cnt1 ? min(a.cnt1[f], a.cap1) : 0;
    const int nb = n0 + n1;
    if (nb > BOX_FAST || nb == 0) return;
    const int* pref = a.pref + (size_t)f * (BOX_FAST + 1);
    const int total = pref[nb];
    if (blockIdx.x * 256 >= total) return;
    const bool use_cells = a.cpref[(size_t)f * (BOX_FAST + 1) + nb] <= CELL_CAP;
    const MBox* table = a.table + (size_t)f * a.tcap;
    const uint64_t* ovl = a.ovl + (size_t)f * BOX_FAST * 4;
    for (int i = threadIdx.x; i < nb; i += 256) {
        s_tab[i] = table[i];
        s_ovl[i][0] = ovl[4 * i + 0]; s_ovl[i][1] = ovl[4 * i + 1];
        s_ovl[i][2] = ovl[4 * i + 2]; s_ovl[i][3] = ovl[4 * i + 3];
    }
    for (int i = threadIdx.x; i <= nb; i += 256) {
        s_pref[i] = pref[i];
        s_cpref[i] = a.cpref[(size_t)f * (BOX_FAST + 1) + i];
    }
    __syncthreads();
    const uint8_t* src = a.in + (size_t)f * a.h * a.pitch;
    uint8_t* dst = a.out + (size_t)f * a.h * a.pitch;
    const uint32_t* cells = a.cells + (size_t)f * CELL_CAP;
    const bool al4 = ((a.pitch & 3) == 0) && (((uintptr_t)a.out & 3) == 0);
    for (int t = blockIdx.x * 256 + threadIdx.x; t < total; t += gridDim.x * 256) {
        const int k = find_box(s_pref, nb, t);
        const MBox& bk = s_tab[k];
        const int q0 = bk.x1 >> 2, nq = ((bk.x2 - 1) >> 2) - q0 + 1;
        const int p = t - s_pref[k];
        const int r = p / nq;
        const int y = bk.y1 + r, xq = (q0 + (p - r * nq)) * 4;
        // pixels of the quad inside box k, minus those a LATER overlapping box contains
        const int lo0 = max(bk.x1 - xq, 0), hi0 = min(bk.x2 - xq, 4);
        unsigned own = ((1u << hi0) - 1u) & ~((1u << lo0) - 1u);
        for (int w = (k + 1) >> 6; w < 4 && own; ++w) {
            uint64_t v = s_ovl[k][w];
            const int lo_bit = k + 1 - (w << 6);
            if (lo_bit > 0) v &= ~((1ULL << lo_bit) - 1ULL);
            while (v && own) {
                const int j = (w << 6) + __ffsll((long long)v) - 1;
                v &= v - 1;
                const MBox& bj = s_tab[j];
                if (y < bj.y1 || y >= bj.y2) continue;
                const int lo = max(bj.x1 - xq, 0), hi = min(bj.x2 - xq, 4);
                if (lo < hi) own &= ~(((1u << hi) - 1u) & ~((1u << lo) - 1u));
            }
        }
        uint32_t col[4] = {0u, 0u, 0u, 0u};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            if (!(own & (1u << e))) continue;
            const int x = xq + e;
            if (use_cells) {
                const int ux = min((int)floor(VD_DMUL((double)(x - bk.x1), bk.fux)), bk.sw - 1);
                const int uy = min((int)floor(VD_DMUL((double)(y - bk.y1), bk.fuy)), bk.sh - 1);
                col[e] = cells[s_cpref[k] + uy * bk.sw + ux];
            } else {
                int yy = y, xx = x;
                apply(bk, yy, xx);
                walk_back(s_tab, s_ovl, k, yy, xx);
                const uint8_t* sp = src + (size_t)yy * a.pitch + xx * 3;
                col[e] = (uint32_t)sp[0] | ((uint32_t)sp[1] << 8) | ((uint32_t)sp[2] << 16);
            }
        }
        if (!own) continue;
        uint8_t* dp = dst + (size_t)y * a.pitch + xq * 3;
        if (own == 15u && al4) {   // 12 bytes = 4 packed RGB pixels
            const uint32_t w0 = col[0] | (col[1] << 24);
            const uint32_t w1 = (col[1] >> 8) | (col[2] << 16);
            const uint32_t w2 = (col[2] >> 16) | (col[3] << 8);
            uint32_t* d32 = (uint32_t*)dp;
            d32[0] = w0; d32[1] = w1; d32[2] = w2;
        } else {
#pragma unroll
            for (int e = 0; e < 4; ++e)
                if (own & (1u << e)) {
                    dp[3 * e] = (uint8_t)col[e]; dp[3 * e + 1] = (uint8_t)(col[e] >> 8);
                    dp[3 * e + 2] = (uint8_t)(col[e] >> 16);
                }
        }
    }
}

}  // namespace

size_t vd_mosaic_table_bytes(int n, int tcap) {
    return (size_t)n * tcap * sizeof(MBox) + (size_t)n * BOX_FAST * 32 + 2 * (size_t)n * (BOX_FAST + 1) * 4 + 16 +
           (size_t)n * CELL_CAP * 4;
}

hipError_t vd_launch_mosaic(const uint8_t* in, uint8_t* out, int n, int h, int w, size_t pitch,
                            const int* cnt0, const int* xy0, int cap0,
                            const int* cnt1, const int* xy1, int cap1, int level, void* table,
                            hipStream_t s) {
    const int vec_ok = (pitch % 16 == 0) && ((uintptr_t)in % 16 == 0) && ((uintptr_t)out % 16 == 0);
    const int tcap = (cnt0 ? cap0 : 0) + (cnt1 ? cap1 : 0);
    char* tail = (char*)table + (size_t)n * tcap * sizeof(MBox);
    char* pre = tail + (size_t)n * BOX_FAST * 32;
    char* cpre = pre + (size_t)n * (BOX_FAST + 1) * 4;
    char* cel = cpre + (size_t)n * (BOX_FAST + 1) * 4;
    cel += (16 - ((uintptr_t)cel & 15)) & 15;
    MosaicArgs a{in, out, n, h, w, pitch, cnt0, xy0, cap0, cnt1, xy1, cap1, level, vec_ok, (MBox*)table, tcap,
                 (uint64_t*)tail, (int*)pre, (int*)cpre, (uint32_t*)cel};
    if (tcap > 0)
        hipLaunchKernelGGL(mosaic_prep_kernel, dim3((tcap + 255) / 256, n), dim3(256), 0, s, a);
    // fast path: copy (~1 MiB per workgroup row of the grid) then owned-pixel gathers
    const size_t fbytes = (size_t)h * pitch;
    const int cblocks = (int)std::min<size_t>(1024, std::max<size_t>(1, fbytes / (64 * 256 * 4)));
    hipLaunchKernelGGL(mosaic_copy_kernel, dim3(cblocks, n), dim3(256), 0, s, a);
    if (tcap > 0) {
        hipLaunchKernelGGL(mosaic_overlap_kernel, dim3(1, n), dim3(256), 0, s, a);
        hipLaunchKernelGGL(mosaic_prefix_kernel, dim3(n), dim3(256), 0, s, a);
        hipLaunchKernelGGL(mosaic_cell_kernel, dim3(CELL_BLOCKS, n), dim3(256), 0, s, a);
        hipLaunchKernelGGL(mosaic_box_kernel, dim3(BOX_BLOCKS, n), dim3(256), 0, s, a);
        // frames with more boxes than the fast path holds
        hipLaunchKernelGGL(mosaic_kernel, dim3((h + ROWS - 1) / ROWS, n), dim3(256), 0, s, a);
    }
    return hipGetLastError();
}
