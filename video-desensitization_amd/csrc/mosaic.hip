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
// Kernels per call (two launches; every output byte is written exactly once):
//  mosaic_cell_kernel  cell_blocks workgroups per frame (option mosaic_cells). Each clips the frame's
//                      boxes and precomputes their resizeNN factors (boxes in call
//                      order: faces first, then plates, combine_detect.py:242-244)
//                      into LDS -- workgroup 0 also writes them, and the cell-count
//                      prefix sums, to the frame's table for the output pass --
//                      builds the overlap graph (bit j of ovl[k] <=> boxes j and k
//                      intersect, by ballots) and the prefix sums of the boxes'
//                      mosaic cell counts (sw*sh); then one thread per mosaic CELL
//                      (ux, uy) of every box: all the pixels of a cell map to the
//                      same point, so the backward walk over earlier boxes and the
//                      3-byte gather run once per cell (level^2 fewer times than
//                      per pixel) into the frame's cell table.
//  mosaic_out_kernel   the output pass, one workgroup per (frame, band of ROWS
//                      rows); every output byte is written once, by 16-B vector
//                      stores in contiguous 1-KB wave spans (details at the kernel).
// HBM traffic = read + write of every frame (2*W*H*3 bytes) + cell gathers (L2).
#include "vd_common.h"
#include "vd_math.h"

#include <algorithm>
#include <type_traits>
#include <cstdlib>

namespace {

constexpr int ROWS = 16;        // rows per output band
constexpr int TB_CAP = 64;      // band-list capacity; fuller bands walk the global table
constexpr int BOX_FAST = 256;   // frames with at most this many boxes get the overlap graph + cell table
constexpr int CELL_CAP = 1 << 18;   // cell-table entries per frame (packed RGB)
constexpr int MAPBOX = 32;      // band boxes the fast path's column maps can name (5 bits)
constexpr int VMAPCAP = 3072;   // vector descriptors per band (row classes x vectors per row)
constexpr int CPLXCAP = 64;     // complex vectors per band with per-pixel entries
constexpr int LCELL = 2048;     // per-band cell-slice entries staged in LDS

struct MBox { int x1, y1, x2, y2; int sw, sh, idx, valid; double fux, fdx, fuy, fdy; };

struct MosaicArgs {
    const uint8_t* in; uint8_t* out; int n, h, w; size_t pitch;
    const int* cnt0; const int* xy0; int cap0;      // list 0 (faces)
    const int* cnt1; const int* xy1; int cap1;      // list 1 (plates, optional)
    int level;
    int vec_ok;                                      // 16-B aligned rows -> vector loads/stores
    MBox* table; int tcap;                           // [n][tcap] prepared boxes
    int* cpref;                                      // [n][BOX_FAST+1] prefix sums of box cells sw*sh
    uint32_t* cells;                                 // [n][CELL_CAP] walked colour per cell
    int map_on;                                      // bit 0: fast path on (option mosaic_map=0 forces the generic
                                                     // path); bit 1: non-temporal output stores, bit 2: loads
};
typedef unsigned mos_u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int frame_boxes(const MosaicArgs& a, int f, int& n0) {
    n0 = a.cnt0 ? min(max(a.cnt0[f], 0), a.cap0) : 0;
    const int n1 = a.cnt1 ? min(max(a.cnt1[f], 0), a.cap1) : 0;
    return n0 + n1;
}

__device__ MBox prep_box(const MosaicArgs& a, int f, int k, int n0) {
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
    return m;
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

// ---- the fused output pass's box form: the clipped rectangle (empty when the box
// is, so neither a band nor a point ever meets it) and sw | sh << 16; resizeNN
// factors are derived where a map is applied, with prep_box's exact operations.
__device__ __forceinline__ int4 clip_rect(const MosaicArgs& a, int f, int k, int n0, uint32_t& sz) {
    const int* src = k < n0 ? a.xy0 + ((size_t)f * a.cap0 + k) * 4 : a.xy1 + ((size_t)f * a.cap1 + (k - n0)) * 4;
    const int x1 = max(0, src[0]), y1 = max(0, src[1]), x2 = min(a.w, src[2]), y2 = min(a.h, src[3]);
    if (!(x2 > x1 && y2 > y1)) { sz = 1u | (1u << 16); return make_int4(0, 0, 0, 0); }   // :150-151
    sz = (uint32_t)max(1, (x2 - x1) / a.level) | ((uint32_t)max(1, (y2 - y1) / a.level) << 16);   // :153-154
    return make_int4(x1, y1, x2, y2);
}

__device__ __forceinline__ bool in_rect(const int4 q, int y, int x) {
    return x >= q.x && x < q.z && y >= q.y && y < q.w;
}

__device__ __forceinline__ double up_factor(int len, int s) {      // resizeNN up:   dst = len, src = s
    return __ddiv_rn(1.0, __ddiv_rn((double)len, (double)s));
}
__device__ __forceinline__ double down_factor(int len, int s) {    // resizeNN down: dst = s, src = len
    return __ddiv_rn(1.0, __ddiv_rn((double)s, (double)len));
}

// apply() of a box given as (rect, sw | sh << 16): bit-identical to prep_box + apply
__device__ __forceinline__ void apply_rect(const int4 q, uint32_t sz, int& y, int& x) {
    const int sw = (int)(sz & 0xFFFFu), sh = (int)(sz >> 16);
    const int bw = q.z - q.x, bh = q.w - q.y;
    const int ux = min((int)floor(VD_DMUL((double)(x - q.x), up_factor(bw, sw))), sw - 1);
    const int dx = min((int)floor(VD_DMUL((double)ux, down_factor(bw, sw))), bw - 1);
    const int uy = min((int)floor(VD_DMUL((double)(y - q.y), up_factor(bh, sh))), sh - 1);
    const int dy = min((int)floor(VD_DMUL((double)uy, down_factor(bh, sh))), bh - 1);
    x = q.x + dx;
    y = q.y + dy;
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
    __shared__ int s_scan[4];
    const int f = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const bool lead = blockIdx.x == 0;            // writes the frame's table for the output pass
    int n0;
    const int nb = frame_boxes(a, f, n0);
    MBox* table = a.table + (size_t)f * a.tcap;
    int* cpref = a.cpref + (size_t)f * (BOX_FAST + 1);
    for (int k = tid; k < nb; k += 256) {
        if (k >= BOX_FAST && !lead) break;
        const MBox m = prep_box(a, f, k, n0);
        if (lead) table[k] = m;
        if (k < BOX_FAST) s_tab[k] = m;
    }
    if (nb > BOX_FAST) { if (lead && tid == 0) cpref[0] = 0; return; }   // uniform over the workgroup
    __syncthreads();
    // overlap graph by ballots: lane l of a wave holds box l + 64*w, the wave tests one box k per step
    {
        int4 rj[4];
        bool vj[4];
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            const int j = w * 64 + lane;
            vj[w] = j < nb && s_tab[j].valid;
            rj[w] = vj[w] ? make_int4(s_tab[j].x1, s_tab[j].y1, s_tab[j].x2, s_tab[j].y2) : make_int4(0, 0, 0, 0);
        }
        for (int k = wid; k < nb; k += 4) {
            const MBox& bk = s_tab[k];
            const bool vk = bk.valid;
            const int kx1 = bk.x1, ky1 = bk.y1, kx2 = bk.x2, ky2 = bk.y2;
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                const int4 q = rj[w];
                const bool hit = vk && vj[w] && (w * 64 + lane) != k && q.x < kx2 && kx1 < q.z && q.y < ky2 && ky1 < q.w;
                const uint64_t bal = __ballot(hit);
                if (lane == 0) s_ovl[k][w] = bal;
            }
        }
    }
    // prefix sums of the boxes' cell counts: wave scans, then the wave totals
    int v = (tid < nb && s_tab[tid].valid) ? s_tab[tid].sw * s_tab[tid].sh : 0;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int u = __shfl_up(v, o);
        if (lane >= o) v += u;
    }
    if (lane == 63) s_scan[wid] = v;
    __syncthreads();
    for (int i = 0; i < wid; ++i) v += s_scan[i];
    if (tid == 0) s_cpref[0] = 0;
    if (tid < nb) s_cpref[tid + 1] = v;
    if (lead) {
        if (tid == 0) cpref[0] = 0;
        if (tid < nb) cpref[tid + 1] = v;
    }
    __syncthreads();
    const int total = s_cpref[nb];
    if (total > CELL_CAP) return;
    const uint8_t* src = a.in + (size_t)f * a.h * a.pitch;
    uint32_t* cells = a.cells + (size_t)f * CELL_CAP;
    for (int t = blockIdx.x * 256 + tid; t < total; t += gridDim.x * 256) {
        const int k = find_box(s_cpref, nb, t);
        const MBox& bk = s_tab[k];
        const int c = t - s_cpref[k];
        const int uy = c / bk.sw, ux = c - uy * bk.sw;
        // apply(bk) of any pixel of this cell: the down-mapped point of (ux, uy)
        int x = bk.x1 + min((int)floor(VD_DMUL((double)ux, bk.fdx)), bk.x2 - bk.x1 - 1);
        int y = bk.y1 + min((int)floor(VD_DMUL((double)uy, bk.fdy)), bk.y2 - bk.y1 - 1);
        walk_back(s_tab, s_ovl, k, y, x);
        const uint8_t* sp = src + (size_t)y * a.pitch + x * 3;
        const uint32_t colour = (uint32_t)sp[0] | ((uint32_t)sp[1] << 8) | ((uint32_t)sp[2] << 16);
        cells[t] = colour;
    }
}

// Backward walk of (y, x) from band entry t (or, on band overflow, over the whole
// table); returns the packed source colour. Out of line: the rare path (cell
// table overflow, > BOX_FAST boxes).
__device__ __forceinline__ uint32_t walk_pixel(const int* band, int t, bool overflow, const MBox* table, int nb,
                                            int y0, const uint8_t* src, size_t pitch, int y, int x) {
    int next_global = nb - 1;
    bool in_band = !overflow;
    if (in_band) {
        for (; t >= 0; --t) {
            const MBox& m = table[band[t]];
            if (inside(m, y, x)) {
                apply(m, y, x);
                if (y < y0) { next_global = m.idx - 1; in_band = false; break; }
            }
        }
    }
    if (!in_band)
        for (int k = next_global; k >= 0; --k) {
            const MBox m = table[k];
            if (m.valid && inside(m, y, x)) apply(m, y, x);
        }
    const uint8_t* sp = src + (size_t)y * pitch + x * 3;
    return (uint32_t)sp[0] | ((uint32_t)sp[1] << 8) | ((uint32_t)sp[2] << 16);
}

// 6-bit pixel mask -> 18-bit byte mask (each pixel's three bytes).
__device__ __forceinline__ unsigned px_to_bytes(unsigned pm) {
    unsigned b = 0;
#pragma unroll
    for (int e = 0; e < 6; ++e) b |= ((pm >> e) & 1u) * (7u << (3 * e));
    return b;
}

// 4-bit byte mask -> 32-bit bit mask (0xFF per selected byte).
__device__ __forceinline__ unsigned byte_mask32(unsigned m4) {
    return ((m4 * 0x204081u) & 0x01010101u) * 0xFFu;
}

// Output pass: every byte of every frame written once (source or mosaic colour).
//
// Fast path (the frame has the cell table, at most MAPBOX boxes meet the band,
// 16-B aligned rows). Prelude, per band: the band's boxes (call order); each
// row's box SET (bit mask) -- rows with the same set have the same ownership
// along x, so the distinct sets ("row classes", usually 1-3 per band) are
// resolved once; the band's rows of every box's cell table copied into LDS; and
// per (row class, 16-B vector of a row) a 32-bit descriptor of the vector's six
// pixels p0..p0+5 (p0 = 16c/3): which are owned (the LAST box containing them),
// and, in the common case of one owner and at most two cell columns, the owner,
// the first column ux0 and the pixel where ux0+1 starts; otherwise an index
// into per-pixel entries. The stream is then nearly branch-free: each wave moves
// contiguous 1-KB spans (16 B per lane, the next four vectors loaded before this
// four are processed and stored); an owned vector costs one descriptor read and
// two cell-colour reads from LDS, its six colours are packed as an 18-byte RGB
// stream, shifted to the vector's byte phase (b0 - 3*p0) with v_alignbyte, and
// merged into the source vector under the owned-byte mask. Rows of classes
// beyond the descriptor capacity scan their box set per vector; bands whose cell
// rows exceed the LDS slice read colours from the global table.
// Generic path (otherwise): 16-B chunks no band box touches are copied, the
// rest take each pixel's owner cell from the global table, or walk when the
// frame has no cell table or the band overflows TB_CAP.
//
// FUSED (option mosaic_fused, default 1): one launch per call, no cell kernel and no
// global cell table. Every workgroup clips its frame's boxes into LDS itself
// (s_box / s_bsz: a few hundred bytes of L2 reads), and the fast path's prelude
// computes the band's cell colours in place of the copy from the cell table: per
// cell of a band box, the down-mapped point, the backward walk over the earlier
// boxes of the frame (the first earlier box containing the point, then from it,
// ...: a box containing a point of box k meets box k, so this is the overlap-graph
// walk of mosaic_cell_kernel), and the 3-byte gather. Bands the fast path does not
// take (more than MAPBOX boxes, cells past the LDS slice, unaligned rows) and frames
// of more than BOX_FAST boxes walk per pixel (the whole box list, from the last box).
// R: rows per band (ROWS, or 24 / 32 with the fused pass: fewer, longer bands for
// batches whose 16-row bands overfill one round of workgroup slots by a little, e.g.
// 32 frames of 720p = 1440 bands on 1280 slots); the LDS cell slice scales with R
template <bool FUSED, int R = ROWS>
__global__ __launch_bounds__(256) void mosaic_out_kernel(MosaicArgs a) {
    constexpr int ROWS = R, LCELL = R < 16 ? 2048 : 128 * R;
    __shared__ int4 s_box[FUSED ? BOX_FAST : 1];       // FUSED: the frame's clipped boxes
    __shared__ uint32_t s_bsz[FUSED ? BOX_FAST : 1];   //        sw | sh << 16
    __shared__ double s_fdx[FUSED ? MAPBOX : 1];       //        down factors of the band boxes
    __shared__ double s_fdy[FUSED ? MAPBOX : 1];
    __shared__ int s_idx[TB_CAP];           // table index of each band box (call order)
    __shared__ int4 s_rect[TB_CAP];         // x1, y1, x2, y2 of each band box
    __shared__ int s_rb[MAPBOX][ROWS];      // LDS cell-slice index of (band box, row)'s cell row
    __shared__ int s_lb[MAPBOX];            // LDS cell-slice base of each band box
    __shared__ int s_uylo[MAPBOX];          // first cell row of each band box inside the band
    __shared__ uint32_t s_lcell[LCELL];     // the band's cell rows, all band boxes
    __shared__ uint32_t s_vmap[VMAPCAP];    // [class][vector] descriptor (see vec_desc)
    __shared__ uint32_t s_cplx[CPLXCAP][3]; // per-pixel entries (owner << 11 | ux, 0xFFFF none) of complex vectors
    __shared__ int s_ncplx;
    __shared__ uint32_t s_cmask[ROWS];      // box set of each row class
    __shared__ int s_rowcls[ROWS];          // row class of each band row (-1: no box)
    __shared__ uint32_t s_pxb[64];          // 6-bit pixel mask -> 18-bit byte mask
    __shared__ double s_fux[MAPBOX];        // resizeNN column factor of each band box
    __shared__ double s_fuy[MAPBOX];
    __shared__ int s_sw[MAPBOX], s_sh[MAPBOX];
    __shared__ int s_cb[MAPBOX];            // cell-table base (cpref) of each band box
    __shared__ int s_ltot, s_ncls, s_bad;
    __shared__ int s_n;
    __shared__ int s_wsum[4];
    const int f = blockIdx.y;
    const int y0 = blockIdx.x * ROWS;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    int n0;
    const int nb = frame_boxes(a, f, n0);
    const MBox* table = a.table + (size_t)f * a.tcap;
    const int* cpref = a.cpref + (size_t)f * (BOX_FAST + 1);
    // FUSED: the frame's boxes fit the LDS table (else per-pixel walks over the raw list)
    const bool use_cells = FUSED ? nb <= BOX_FAST : (nb <= BOX_FAST && cpref[nb] <= CELL_CAP);
    if constexpr (FUSED) {
        if (use_cells)
            for (int k = tid; k < nb; k += 256) {
                uint32_t sz;
                s_box[k] = clip_rect(a, f, k, n0, sz);
                s_bsz[k] = sz;
            }
    }
    if (tid == 0) s_n = 0;
    __syncthreads();
    // box k of the frame as (rect, sw | sh << 16); invalid boxes have an empty rect
    auto box_rect = [&](int k, uint32_t& sz) -> int4 {
        if constexpr (FUSED) {
            if (use_cells) { sz = s_bsz[k]; return s_box[k]; }
            return clip_rect(a, f, k, n0, sz);
        } else {
            const MBox& m = table[k];
            sz = (uint32_t)m.sw | ((uint32_t)m.sh << 16);
            return m.valid ? make_int4(m.x1, m.y1, m.x2, m.y2) : make_int4(0, 0, 0, 0);
        }
    };
    // ordered compaction of the boxes intersecting rows [y0, y0+ROWS)
    for (int base = 0; base < nb; base += 256) {
        const int k = base + tid;
        bool hit = false;
        int4 q = make_int4(0, 0, 0, 0);
        if (k < nb) {
            uint32_t sz;
            q = box_rect(k, sz);
            hit = q.z > q.x && q.y < y0 + ROWS && q.w > y0;
        }
        const uint64_t bal = __ballot(hit);
        const int wpre = __popcll(bal & ((1ULL << lane) - 1ULL));
        if (lane == 0) s_wsum[wid] = __popcll(bal);
        __syncthreads();
        int off = s_n;
        for (int i = 0; i < wid; ++i) off += s_wsum[i];
        if (hit && off + wpre < TB_CAP) {
            s_idx[off + wpre] = k;
            s_rect[off + wpre] = q;
        }
        __syncthreads();
        if (tid == 0) s_n += s_wsum[0] + s_wsum[1] + s_wsum[2] + s_wsum[3];
        __syncthreads();
    }
    const bool overflow = s_n > TB_CAP;
    const int nt = min(s_n, TB_CAP);
    const int rows = min(ROWS, a.h - y0);

    const uint8_t* src = a.in + (size_t)f * a.h * a.pitch;
    uint8_t* dst = a.out + (size_t)f * a.h * a.pitch;
    const int row_bytes = a.w * 3;
    const uint32_t* cells = a.cells + (size_t)f * CELL_CAP;

    bool fast = use_cells && !overflow && a.vec_ok && nt <= MAPBOX && (a.map_on & 1);
    if (fast) {
        // wave 0, per band box t: the band's slice of its cell rows [uy_lo, uy_hi]
        // (exclusive prefix sum of their cell counts); sw must fit the map's 11 bits
        if (wid == 0) {
            int t = lane, nc = 0, bad = 0;
            if (t < nt) {
                int sw, sh, y1, y2;
                double fux, fuy;
                if constexpr (FUSED) {
                    const int4 q = s_rect[t];
                    const uint32_t sz = s_bsz[s_idx[t]];
                    sw = (int)(sz & 0xFFFFu);
                    sh = (int)(sz >> 16);
                    y1 = q.y;
                    y2 = q.w;
                    fux = up_factor(q.z - q.x, sw);
                    fuy = up_factor(q.w - q.y, sh);
                    s_fdx[t] = down_factor(q.z - q.x, sw);
                    s_fdy[t] = down_factor(q.w - q.y, sh);
                } else {
                    const MBox& m = table[s_idx[t]];
                    sw = m.sw; sh = m.sh; y1 = m.y1; y2 = m.y2; fux = m.fux; fuy = m.fuy;
                    s_cb[t] = cpref[m.idx];
                }
                const int ya = max(y0, y1), yb = min(y0 + rows, y2) - 1;
                const int ulo = min((int)floor(VD_DMUL((double)(ya - y1), fuy)), sh - 1);
                const int uhi = min((int)floor(VD_DMUL((double)(yb - y1), fuy)), sh - 1);
                nc = (uhi - ulo + 1) * sw;
                bad = sw > 2047;
                s_uylo[t] = ulo;
                s_fux[t] = fux;
                s_fuy[t] = fuy;
                s_sw[t] = sw;
                s_sh[t] = sh;
            }
            int v = nc;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const int u = __shfl_up(v, o);
                if (lane >= o) v += u;
            }
            if (t < nt) s_lb[t] = v - nc;
            const uint64_t anybad = __ballot(bad);
            if (lane == 63) s_ltot = v;
            // row sets (lane r <-> band row r), then their distinct classes
            uint32_t rm = 0;
            if (lane < ROWS && lane < rows)
                for (int q = 0; q < nt; ++q)
                    if (y0 + lane >= s_rect[q].y && y0 + lane < s_rect[q].w) rm |= 1u << q;
            int cls = -1, ncls = 0;
            for (int r = 0; r < ROWS; ++r) {          // wave-uniform walk over the rows
                const uint32_t mr = __shfl(rm, r);
                if (!mr) continue;
                int found = -1;
                for (int k = 0; k < ncls; ++k) if (s_cmask[k] == mr) { found = k; break; }
                if (found < 0) {
                    found = ncls;
                    if (ncls < ROWS && lane == 0) s_cmask[ncls] = mr;
                    ++ncls;
                    __builtin_amdgcn_wave_barrier();
                }
                if (lane == r) cls = found;
            }
            if (lane < ROWS) s_rowcls[lane] = cls;
            if (lane == 0) { s_ncls = ncls; s_bad = anybad != 0; s_ncplx = 0; }
        }
        if (tid < 64) s_pxb[tid] = px_to_bytes(tid);
        __syncthreads();
        fast = !s_bad && (!FUSED || s_ltot <= LCELL);   // FUSED: no global cell table to fall back on
    }

    if (!fast) {
        const int nchunk = (row_bytes + 15) >> 4;
        const bool cell_owner = !FUSED && use_cells && !overflow;
        for (int i = tid; i < rows * nchunk; i += 256) {
            const int r = i / nchunk, c = i - r * nchunk;
            const int y = y0 + r;
            const uint8_t* srow = src + (size_t)y * a.pitch;
            uint8_t* drow = dst + (size_t)y * a.pitch;
            const int b0 = c << 4;
            const int bend = min(b0 + 16, row_bytes);
            const int px0 = b0 / 3, px1 = (bend - 1) / 3;
            bool touched = overflow;
            for (int t = 0; t < nt && !touched; ++t) {
                const int4 q = s_rect[t];
                touched = y >= q.y && y < q.w && px1 >= q.x && px0 < q.z;
            }
            if (!touched && bend - b0 == 16 && a.vec_ok) {
                *(uint4*)(drow + b0) = *(const uint4*)(srow + b0);
                continue;
            }
            if (!touched) {
                for (int bb = b0; bb < bend; ++bb) drow[bb] = srow[bb];
                continue;
            }
            int lastx = -1;
            uint32_t cv = 0;
            for (int bb = b0; bb < bend; ++bb) {
                const int x = bb / 3, ch = bb - 3 * x;
                if (x != lastx) {
                    lastx = x;
                    if (FUSED) {
                    } else if (cell_owner) {
                        int t = nt - 1;
                        for (; t >= 0; --t) {
                            const int4 q = s_rect[t];
                            if (y >= q.y && y < q.w && x >= q.x && x < q.z) break;
                        }
                        if (t < 0) {
                            cv = (uint32_t)srow[3 * x] | ((uint32_t)srow[3 * x + 1] << 8) | ((uint32_t)srow[3 * x + 2] << 16);
                        } else {
                            const MBox& m = table[s_idx[t]];
                            const int ux = min((int)floor(VD_DMUL((double)(x - m.x1), m.fux)), m.sw - 1);
                            const int uy = min((int)floor(VD_DMUL((double)(y - m.y1), m.fuy)), m.sh - 1);
                            cv = cells[cpref[m.idx] + uy * m.sw + ux];
                        }
                    } else {
                        cv = walk_pixel(s_idx, nt - 1, overflow, table, nb, y0, src, a.pitch, y, x);
                    }
                    if constexpr (FUSED) {     // the whole list, last box first (box_rect: LDS or raw)
                        int yy = y, xx = x;
                        for (int k = nb - 1; k >= 0; --k) {
                            uint32_t sz;
                            const int4 q = box_rect(k, sz);
                            if (in_rect(q, yy, xx)) apply_rect(q, sz, yy, xx);
                        }
                        const uint8_t* sp = src + (size_t)yy * a.pitch + xx * 3;
                        cv = (uint32_t)sp[0] | ((uint32_t)sp[1] << 8) | ((uint32_t)sp[2] << 16);
                    }
                }
                drow[bb] = (uint8_t)(cv >> (8 * ch));
            }
        }
        return;
    }

    const bool lcell_ok = s_ltot <= LCELL;        // else cells are read from the global table
    const int vpr = (int)(a.pitch >> 4);          // 16-B vectors per row (pitch % 16 == 0 here)
    const int dmax = min(ROWS, VMAPCAP / vpr);    // row classes with a vector map
    // per (band box, row): index of the box's cell row (LDS slice or global table)
    for (int i = tid; i < MAPBOX * ROWS; i += 256) {   // (entries past nt: 0, read by unowned pixels)
        const int t = i / ROWS, r = i - t * ROWS;
        const int y = y0 + r;
        int v = 0;
        if (t < nt && y >= s_rect[t].y && y < s_rect[t].w) {
            const int uy = min((int)floor(VD_DMUL((double)(y - s_rect[t].y), s_fuy[t])), s_sh[t] - 1);
            v = lcell_ok ? s_lb[t] + (uy - s_uylo[t]) * s_sw[t] : s_cb[t] + uy * s_sw[t];
        }
        s_rb[t][r] = v;
    }
    // the band's cell rows of every box: contiguous in the global cell table, or
    // (FUSED) walked and gathered here, one thread per cell
    if (FUSED && lcell_ok && (a.map_on & 16)) {
        // option mosaic_gather: a thread's cells walked first (LDS only), then all their
        // source-pixel loads issued together -- one global latency per pass, not one per cell
        constexpr int G = 8;
        for (int i0 = tid; i0 < s_ltot; i0 += 256 * G) {
            const uint8_t* sp[G];
#pragma unroll
            for (int u = 0; u < G; ++u) {
                const int i = i0 + 256 * u;
                sp[u] = nullptr;
                if (i < s_ltot) {
                    int t = 0;
                    while (t + 1 < nt && s_lb[t + 1] <= i) ++t;
                    const int c = i - s_lb[t], sw = s_sw[t];
                    const int cr = c / sw, ux = c - cr * sw, uy = s_uylo[t] + cr;
                    const int4 q = s_rect[t];
                    int x = q.x + min((int)floor(VD_DMUL((double)ux, s_fdx[t])), q.z - q.x - 1);
                    int y = q.y + min((int)floor(VD_DMUL((double)uy, s_fdy[t])), q.w - q.y - 1);
                    for (int j = s_idx[t] - 1; j >= 0; --j) {
                        const int4 r = s_box[j];
                        if (in_rect(r, y, x)) apply_rect(r, s_bsz[j], y, x);
                    }
                    sp[u] = src + (size_t)y * a.pitch + x * 3;
                }
            }
            uint32_t cv[G];
#pragma unroll
            for (int u = 0; u < G; ++u)
                cv[u] = sp[u] ? (uint32_t)sp[u][0] | ((uint32_t)sp[u][1] << 8) | ((uint32_t)sp[u][2] << 16) : 0u;
#pragma unroll
            for (int u = 0; u < G; ++u)
                if (sp[u]) s_lcell[i0 + 256 * u] = cv[u];
        }
    } else if (lcell_ok)
        for (int i = tid; i < s_ltot; i += 256) {
            int t = 0;
            while (t + 1 < nt && s_lb[t + 1] <= i) ++t;
            if constexpr (FUSED) {
                const int c = i - s_lb[t], sw = s_sw[t];
                const int cr = c / sw, ux = c - cr * sw, uy = s_uylo[t] + cr;
                const int4 q = s_rect[t];
                // any pixel of cell (ux, uy) maps to this point under box t
                int x = q.x + min((int)floor(VD_DMUL((double)ux, s_fdx[t])), q.z - q.x - 1);
                int y = q.y + min((int)floor(VD_DMUL((double)uy, s_fdy[t])), q.w - q.y - 1);
                for (int j = s_idx[t] - 1; j >= 0; --j) {
                    const int4 r = s_box[j];
                    if (in_rect(r, y, x)) apply_rect(r, s_bsz[j], y, x);
                }
                const uint8_t* sp = src + (size_t)y * a.pitch + x * 3;
                s_lcell[i] = (uint32_t)sp[0] | ((uint32_t)sp[1] << 8) | ((uint32_t)sp[2] << 16);
            } else {
                s_lcell[i] = cells[s_cb[t] + s_uylo[t] * s_sw[t] + (i - s_lb[t])];
            }
        }
    // vector maps of the first dmax row classes (rows of later classes scan per vector):
    // one descriptor per 16-B vector = pixels p0..p0+5 of the row
    //   bits 0-5 owned pixels; kind (bits 25-26) 0: one owner t (bits 6-10), pixels
    //   before the split s (bits 22-24) in cell column ux0 (bits 11-21), the rest in
    //   ux0 + 1; 1: per-pixel entries in s_cplx[bits 6-21]; 2: scan per pixel.
    const int ncls = min(s_ncls, dmax);
    for (int k = 0; k < ncls; ++k) {
        const uint32_t mk0 = s_cmask[k];
        for (int c = tid; c < vpr; c += 256) {
            const int b0 = c << 4;
            uint32_t d = 0;
            if (b0 < row_bytes) {
                const int p0 = b0 / 3, np = min(6, a.w - p0);
                // owners: the class's boxes, last first, each claiming its x-range of the six pixels
                int own[6];
#pragma unroll
                for (int e = 0; e < 6; ++e) own[e] = 0;
                const unsigned full = (1u << np) - 1u;
                unsigned todo = full;
                uint32_t mk = mk0;
                while (mk && todo) {
                    const int t = 31 - __clz((int)mk);
                    mk ^= 1u << t;
                    const int4 q = s_rect[t];
                    const int lo = max(q.x - p0, 0), hi = min(q.z - p0, np);
                    if (lo >= hi) continue;
                    const unsigned bits = ((1u << hi) - 1u) & ~((1u << lo) - 1u) & todo;
                    todo &= ~bits;
#pragma unroll
                    for (int e = 0; e < 6; ++e)
                        if (bits & (1u << e)) own[e] = t;
                }
                const unsigned pm = full & ~todo;
                const int t0 = pm ? own[__ffs(pm) - 1] : 0;
                bool one = true;
#pragma unroll
                for (int e = 0; e < 6; ++e)
                    if ((pm & (1u << e)) && own[e] != t0) one = false;
                unsigned ent[6];
                if (one) {
                    const int x1 = s_rect[t0].x, swm = s_sw[t0] - 1;
                    const double fx = s_fux[t0];
#pragma unroll
                    for (int e = 0; e < 6; ++e)
                        ent[e] = (pm & (1u << e))
                                     ? (unsigned)((t0 << 11) | min((int)floor(VD_DMUL((double)(p0 + e - x1), fx)), swm))
                                     : 0xFFFFu;
                } else {
#pragma unroll
                    for (int e = 0; e < 6; ++e) {
                        ent[e] = 0xFFFFu;
                        if (pm & (1u << e)) {
                            const int t = own[e];
                            const int ux = min((int)floor(VD_DMUL((double)(p0 + e - s_rect[t].x), s_fux[t])), s_sw[t] - 1);
                            ent[e] = (unsigned)((t << 11) | ux);
                        }
                    }
                }
                if (pm) {
                    // one owner, at most two consecutive cell columns, split monotone
                    unsigned ux0 = 0xFFFFu, split = 6;
                    if (one) {
#pragma unroll
                        for (int e = 5; e >= 0; --e)
                            if (pm & (1u << e)) ux0 = ent[e] & 2047u;          // first owned pixel's column
#pragma unroll
                        for (int e = 0; e < 6; ++e) {
                            if (!(pm & (1u << e))) continue;
                            const unsigned ux = ent[e] & 2047u;
                            if (ux == ux0 + 1 && split == 6) split = e;
                            else if (ux != ux0 && ux != ux0 + 1) one = false;
                        }
                    }
                    if (one) {
                        d = pm | ((unsigned)t0 << 6) | (ux0 << 11) | (split << 22);
                    } else {
                        const int ci = atomicAdd(&s_ncplx, 1);
                        if (ci < CPLXCAP) {
                            s_cplx[ci][0] = ent[0] | (ent[1] << 16);
                            s_cplx[ci][1] = ent[2] | (ent[3] << 16);
                            s_cplx[ci][2] = ent[4] | (ent[5] << 16);
                            d = pm | ((unsigned)ci << 6) | (1u << 25);
                        } else {
                            d = pm | (2u << 25);
                        }
                    }
                }
            }
            s_vmap[k * vpr + c] = d;
        }
    }
    __syncthreads();

    const int nvec = rows * vpr;
    const uint4* s4 = (const uint4*)(src + (size_t)y0 * a.pitch);
    uint4* d4 = (uint4*)(dst + (size_t)y0 * a.pitch);

    // vector (r, c) = bytes [16c, 16c+16) of band row r. LDS: cell colours from the
    // band's LDS slice (no global access, so no vmcnt wait inside); otherwise from
    // the global cell table.
    auto process = [&](uint4& v, int r, int c, auto lds) {
        constexpr bool LDS = decltype(lds)::value;
        const int k = s_rowcls[r];
        const int b0 = c << 4;
        if (k < 0 || b0 >= row_bytes) return;      // no box on this row / row padding
        const int p0 = b0 / 3, phase = b0 - 3 * p0;
        const int np = min(6, a.w - p0);
        auto colour = [&](int idx) -> uint32_t {
            if constexpr (LDS) return s_lcell[min(idx, LCELL - 1)];
            else return cells[idx];
        };
        uint32_t col[6];
        unsigned pm = 0;
        const uint32_t d = k < dmax ? s_vmap[k * vpr + c] : (2u << 25);
        const unsigned kind = d >> 25;
        if (kind == 0) {                           // one owner, <= 2 cell columns
            pm = d & 63u;
            if (!pm) return;
            const int t = (d >> 6) & 31, ux0 = (d >> 11) & 2047, split = (d >> 22) & 7;
            const int rb = s_rb[t][r] + ux0;
            const uint32_t c0 = colour(rb), c1 = split < 6 ? colour(rb + 1) : c0;
#pragma unroll
            for (int e = 0; e < 6; ++e) col[e] = e < split ? c0 : c1;
        } else {
            unsigned uu[6];
            if (kind == 1) {                       // per-pixel entries
                pm = d & 63u;
                const int ci = (d >> 6) & 0xFFFF;
                const uint32_t q0 = s_cplx[ci][0], q1 = s_cplx[ci][1], q2 = s_cplx[ci][2];
                uu[0] = q0 & 0xFFFFu; uu[1] = q0 >> 16; uu[2] = q1 & 0xFFFFu;
                uu[3] = q1 >> 16; uu[4] = q2 & 0xFFFFu; uu[5] = q2 >> 16;
            } else {                               // scan the row class's box set
#pragma unroll
                for (int e = 0; e < 6; ++e) {
                    uu[e] = 0xFFFFu;
                    if (e >= np) continue;
                    const int x = p0 + e;
                    uint32_t mk = s_cmask[k];
                    while (mk) {
                        const int t = 31 - __clz((int)mk);
                        mk ^= 1u << t;
                        const int4 q = s_rect[t];
                        if (x >= q.x && x < q.z) {
                            const int ux = min((int)floor(VD_DMUL((double)(x - q.x), s_fux[t])), s_sw[t] - 1);
                            uu[e] = (unsigned)((t << 11) | ux);
                            pm |= 1u << e;
                            break;
                        }
                    }
                }
                if (!pm) return;
            }
#pragma unroll
            for (int e = 0; e < 6; ++e) {
                const unsigned u = uu[e];
                const int idx = s_rb[min(u >> 11, (unsigned)MAPBOX - 1)][r] + (int)(u & 2047u);
                col[e] = u == 0xFFFFu ? 0u : colour(idx);
            }
        }
        // 18-byte RGB stream of the six pixels, shifted to the vector's phase
        const uint32_t w0 = col[0] | (col[1] << 24), w1 = (col[1] >> 8) | (col[2] << 16);
        const uint32_t w2 = (col[2] >> 16) | (col[3] << 8), w3 = col[4] | (col[5] << 24), w4 = col[5] >> 8;
        const unsigned sh = phase;
        const uint32_t m0 = __builtin_amdgcn_alignbyte(w1, w0, sh), m1 = __builtin_amdgcn_alignbyte(w2, w1, sh);
        const uint32_t m2 = __builtin_amdgcn_alignbyte(w3, w2, sh), m3 = __builtin_amdgcn_alignbyte(w4, w3, sh);
        const unsigned bm = s_pxb[pm] >> phase;
        const uint32_t k0 = byte_mask32(bm & 15u), k1 = byte_mask32((bm >> 4) & 15u);
        const uint32_t k2 = byte_mask32((bm >> 8) & 15u), k3 = byte_mask32((bm >> 12) & 15u);
        v.x = (v.x & ~k0) | (m0 & k0);
        v.y = (v.y & ~k1) | (m1 & k1);
        v.z = (v.z & ~k2) | (m2 & k2);
        v.w = (v.w & ~k3) | (m3 & k3);
    };
    auto advance = [&](int& r, int& c) {           // (r, c) += 256 vectors
        c += 256;
        while (c >= vpr) { c -= vpr; ++r; }
    };
    // Software-pipelined stream: the next four vectors are loaded before this
    // four are processed and stored, so the stores of one step never sit ahead
    // of the loads the next step waits for.
    auto stream = [&](auto lds) {
        int r = tid / vpr, c = tid - (tid / vpr) * vpr;
        int j = tid;
        uint4 v0{}, v1{}, v2{}, v3{};
        const bool nt_st = a.map_on & 2, nt_ld = a.map_on & 4;
        auto ld = [&](int jj) -> uint4 {
            if (nt_ld) return __builtin_bit_cast(uint4, __builtin_nontemporal_load((const mos_u32x4*)(s4 + jj)));
            return s4[jj];
        };
        auto st = [&](int jj, const uint4& v) {
            if (nt_st) __builtin_nontemporal_store(__builtin_bit_cast(mos_u32x4, v), (mos_u32x4*)(d4 + jj));
            else d4[jj] = v;
        };
        auto load4 = [&](int jj, uint4& x0, uint4& x1, uint4& x2, uint4& x3) {
            if (jj < nvec) x0 = ld(jj);
            if (jj + 256 < nvec) x1 = ld(jj + 256);
            if (jj + 512 < nvec) x2 = ld(jj + 512);
            if (jj + 768 < nvec) x3 = ld(jj + 768);
        };
        load4(j, v0, v1, v2, v3);
        for (; j < nvec; j += 4 * 256) {
            uint4 n0{}, n1{}, n2{}, n3{};
            load4(j + 1024, n0, n1, n2, n3);
            const bool h1 = j + 256 < nvec, h2 = j + 512 < nvec, h3 = j + 768 < nvec;
            int r1 = r, c1 = c;
            advance(r1, c1);
            int r2 = r1, c2 = c1;
            advance(r2, c2);
            int r3 = r2, c3 = c2;
            advance(r3, c3);
            if (nt) {
                process(v0, r, c, lds);
                if (h1) process(v1, r1, c1, lds);
                if (h2) process(v2, r2, c2, lds);
                if (h3) process(v3, r3, c3, lds);
            }
            st(j, v0);
            if (h1) st(j + 256, v1);
            if (h2) st(j + 512, v2);
            if (h3) st(j + 768, v3);
            r = r3; c = c3;
            advance(r, c);
            v0 = n0; v1 = n1; v2 = n2; v3 = n3;
        }
    };
    if (lcell_ok) stream(std::true_type{});
    else stream(std::false_type{});
}

}  // namespace

// Band height of the fused output pass (option mosaic_rows: 4 / 8 / 16 / 24 / 32; 0 =
// auto). Measured (profiles/r06_mosaic_rows.txt): bands of ~30-45 KB of pixels stream
// best -- 8 rows at 720p / 1080p (1080p blur 0.52 -> 0.55 of the HBM peak), 4 rows at 4K
// (0.50 -> 0.64); 24- / 32-row bands are slower everywhere (more row classes than the
// vector maps hold take the per-pixel scan, and the prelude grows).
static int mosaic_rows_for(int w, int opt) {
    if (opt == 4 || opt == 8 || opt == ROWS || opt == 24 || opt == 32) return opt;
    return w * 3 >= 8192 ? 4 : 8;
}

size_t vd_mosaic_table_bytes(int n, int tcap) {
    return (size_t)n * tcap * sizeof(MBox) + (size_t)n * (BOX_FAST + 1) * 4 + 16 +
           (size_t)n * CELL_CAP * 4;
}

hipError_t vd_launch_mosaic(const uint8_t* in, uint8_t* out, int n, int h, int w, size_t pitch,
                            const int* cnt0, const int* xy0, int cap0,
                            const int* cnt1, const int* xy1, int cap1, int level, void* table,
                            int stages, int map_on, int cell_blocks, hipStream_t s) {
    if (n <= 0 || h <= 0 || w <= 0) return hipSuccess;
    cell_blocks = std::min(std::max(cell_blocks, 1), 256);
    const int vec_ok = (pitch % 16 == 0) && ((uintptr_t)in % 16 == 0) && ((uintptr_t)out % 16 == 0);
    const int tcap = (cnt0 ? cap0 : 0) + (cnt1 ? cap1 : 0);
    char* cpre = (char*)table + (size_t)n * tcap * sizeof(MBox);
    char* cel = cpre + (size_t)n * (BOX_FAST + 1) * 4;
    cel += (16 - ((uintptr_t)cel & 15)) & 15;
    MosaicArgs a{in, out, n, h, w, pitch, cnt0, xy0, cap0, cnt1, xy1, cap1, level, vec_ok, (MBox*)table, tcap,
                 (int*)cpre, (uint32_t*)cel, 1};
    a.map_on = map_on;
    if (stages & 1) hipLaunchKernelGGL(mosaic_cell_kernel, dim3(cell_blocks, n), dim3(256), 0, s, a);
    if (stages & 2) hipLaunchKernelGGL(mosaic_out_kernel<false>, dim3((h + ROWS - 1) / ROWS, n), dim3(256), 0, s, a);
    if (stages & 8) {
        const int r = mosaic_rows_for(w, map_on >> 8);
        if (r == 8) hipLaunchKernelGGL((mosaic_out_kernel<true, 8>), dim3((h + 7) / 8, n), dim3(256), 0, s, a);
        else if (r == 4) hipLaunchKernelGGL((mosaic_out_kernel<true, 4>), dim3((h + 3) / 4, n), dim3(256), 0, s, a);
        else if (r == 32) hipLaunchKernelGGL((mosaic_out_kernel<true, 32>), dim3((h + 31) / 32, n), dim3(256), 0, s, a);
        else if (r == 24) hipLaunchKernelGGL((mosaic_out_kernel<true, 24>), dim3((h + 23) / 24, n), dim3(256), 0, s, a);
        else hipLaunchKernelGGL((mosaic_out_kernel<true, ROWS>), dim3((h + ROWS - 1) / ROWS, n), dim3(256), 0, s, a);
    }
    return hipGetLastError();
}
