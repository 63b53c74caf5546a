// jpeg_enc.hip — device stage of the JPEG frame encode (host stage: jpeg_enc.cpp).
//
// libjpeg-turbo's compressor with its defaults [ext], as cv2.imwrite runs it on
// every processed frame (combine_detect.py:174-180, :259-262), restated
// bit-exactly (oracle/jpeg_enc.py, pinned byte for byte against Pillow's
// libjpeg-turbo):
//   jpeg_fdct_kernel   8 lanes per 8x8 block of one component. Lane r forms
//                      row r of the block straight from the RGB frame: the
//                      jccolor.c fixed-point RGB->YCbCr of each pixel, the
//                      jcsample.c box average with its alternating bias for
//                      subsampled chroma, edge replication (jcprepct.c /
//                      expand_right_edge) as coordinate clamping; then the
//                      jfdctint.c ISLOW row pass (lane = row), an LDS
//                      transpose, the column pass (lane = column) and the
//                      jcdctmgr.c reciprocal quantisation; the block's 64
//                      coefficients (natural order, int16) leave as one
//                      128-byte store of 8 lanes.
// The Huffman stage (sequential per scan) runs on host threads over these blocks.
#include "vd_common.h"

namespace {

constexpr int CONST_BITS = 13, PASS1_BITS = 2;
constexpr int BLK_PER_WG = 32;                          // 8 lanes per block, 256 threads

__device__ __forceinline__ int descale(int x, int n) { return (x + (1 << (n - 1))) >> n; }

// jccolor.c rgb_ycc_convert (SCALEBITS 16, tables folded into constants)
__device__ __forceinline__ int ycc(int c, int r, int g, int b) {
    if (c == 0) return (19595 * r + 38470 * g + 7471 * b + 32768) >> 16;
    if (c == 1) return (-11059 * r - 21709 * g + 32768 * b + (128 << 16) + 32767) >> 16;
    return (32768 * r - 27439 * g - 5329 * b + (128 << 16) + 32767) >> 16;
}

__device__ __forceinline__ int pix(const JpegEncArgs& a, const uint8_t* f, int c, int y, int x) {
    y = y < a.h ? y : a.h - 1;
    x = x < a.w ? x : a.w - 1;
    const uint8_t* p = f + (size_t)y * a.pitch + (size_t)x * 3;
    return ycc(c, p[0], p[1], p[2]);
}

// component sample (sy, sx) before the level shift
__device__ __forceinline__ int sample(const JpegEncArgs& a, const uint8_t* f, int c, int sy, int sx) {
    if (c == 0 || (a.hl == 1 && a.vl == 1)) return pix(a, f, c, sy, sx);
    const int rows = (a.h + a.vl - 1) / a.vl;          // downsampled rows that hold image data
    const int cy = sy < rows ? sy : rows - 1;          // below them: the last one replicated
    const int fx = sx * a.hl;
    if (a.vl == 1)                                      // h2v1: bias 0, 1, 0, 1, ...
        return (pix(a, f, c, cy, fx) + pix(a, f, c, cy, fx + 1) + (sx & 1)) >> 1;
    const int fy = cy * 2;                              // h2v2: bias 1, 2, 1, 2, ...
    return (pix(a, f, c, fy, fx) + pix(a, f, c, fy, fx + 1) + pix(a, f, c, fy + 1, fx) +
            pix(a, f, c, fy + 1, fx + 1) + 1 + (sx & 1)) >> 2;
}

// one jpeg_fdct_islow pass over 8 values (pass 1: rows, LEFT_SHIFT; pass 2: columns)
template <bool FIRST>
__device__ __forceinline__ void fdct8(int (&d)[8]) {
    const int t0 = d[0] + d[7], t7 = d[0] - d[7], t1 = d[1] + d[6], t6 = d[1] - d[6];
    const int t2 = d[2] + d[5], t5 = d[2] - d[5], t3 = d[3] + d[4], t4 = d[3] - d[4];
    const int t10 = t0 + t3, t13 = t0 - t3, t11 = t1 + t2, t12 = t1 - t2;
    constexpr int SH = FIRST ? CONST_BITS - PASS1_BITS : CONST_BITS + PASS1_BITS;
    if (FIRST) {
        d[0] = (t10 + t11) * (1 << PASS1_BITS);
        d[4] = (t10 - t11) * (1 << PASS1_BITS);
    } else {
        d[0] = descale(t10 + t11, PASS1_BITS);
        d[4] = descale(t10 - t11, PASS1_BITS);
    }
    int z1 = (t12 + t13) * 4433;                       // FIX_0_541196100
    d[2] = descale(z1 + t13 * 6270, SH);               // FIX_0_765366865
    d[6] = descale(z1 - t12 * 15137, SH);              // FIX_1_847759065
    z1 = t4 + t7;
    int z2 = t5 + t6, z3 = t4 + t6, z4 = t5 + t7;
    const int z5 = (z3 + z4) * 9633;                   // FIX_1_175875602
    const int a4 = t4 * 2446, a5 = t5 * 16819, a6 = t6 * 25172, a7 = t7 * 12299;
    z1 *= -7373;                                       // FIX_0_899976223
    z2 *= -20995;                                      // FIX_2_562915447
    z3 = z3 * -16069 + z5;                             // FIX_1_961570560
    z4 = z4 * -3196 + z5;                              // FIX_0_390180644
    d[7] = descale(a4 + z1 + z3, SH);
    d[5] = descale(a5 + z2 + z4, SH);
    d[3] = descale(a6 + z2 + z3, SH);
    d[1] = descale(a7 + z1 + z4, SH);
}

__global__ __launch_bounds__(256) void jpeg_fdct_kernel(JpegEncArgs a) {
    __shared__ int tile[BLK_PER_WG][8][9];
    __shared__ __attribute__((aligned(16))) int16_t outb[BLK_PER_WG][64];
    const int lb = threadIdx.x >> 3, lane = threadIdx.x & 7;
    const long g = (long)blockIdx.x * BLK_PER_WG + lb;
    const long total = (long)a.n * a.blocks_per_frame;
    const bool valid = g < total;
    const long gg = valid ? g : total - 1;
    const int frame = (int)(gg / a.blocks_per_frame);
    const int local = (int)(gg - (long)frame * a.blocks_per_frame);
    const int c = local >= a.cblk[2] ? 2 : (local >= a.cblk[1] ? 1 : 0);
    const int bi = local - a.cblk[c];
    const int by = bi / a.bw[c], bx = bi - by * a.bw[c];
    const uint8_t* f = a.src + (size_t)frame * a.h * a.pitch;
    // row pass: lane = row
    int d[8];
#pragma unroll
    for (int x = 0; x < 8; ++x) d[x] = sample(a, f, c, by * 8 + lane, bx * 8 + x) - 128;
    fdct8<true>(d);
#pragma unroll
    for (int x = 0; x < 8; ++x) tile[lb][lane][x] = d[x];
    __syncthreads();
    // column pass: lane = column, then quantise (natural index r * 8 + lane)
#pragma unroll
    for (int y = 0; y < 8; ++y) d[y] = tile[lb][y][lane];
    fdct8<false>(d);
    const int t = c == 0 ? 0 : 1;
#pragma unroll
    for (int y = 0; y < 8; ++y) {
        const int k = y * 8 + lane;
        const int x = d[y];
        const unsigned m = ((unsigned)(x < 0 ? -x : x) + a.corr[t * 64 + k]) * (unsigned)a.recip[t * 64 + k];
        const int q = (int)(m >> a.shift[t * 64 + k]);
        outb[lb][k] = (int16_t)(x < 0 ? -q : q);
    }
    __syncthreads();
    if (valid) *(uint4*)(a.coef + g * 64 + lane * 8) = *(const uint4*)&outb[lb][lane * 8];
}

}  // namespace

hipError_t vd_launch_jpeg_fdct(const JpegEncArgs& a, hipStream_t s) {
    const long total = (long)a.n * a.blocks_per_frame;
    if (total <= 0) return hipSuccess;
    hipLaunchKernelGGL(jpeg_fdct_kernel, dim3((unsigned)((total + BLK_PER_WG - 1) / BLK_PER_WG)), dim3(256), 0, s, a);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Entropy stage on the device (jchuff.c encode_one_block over the interleaved
// scan, the same arithmetic as jpeg_enc.cpp's host coder, byte-identical output):
//   jpeg_hsize_kernel  one thread per scan unit: DC difference (predecessor of the
//                      same component in scan order; dummy blocks carry the DC of
//                      the block before them in their MCU, jccoefct.c) and the
//                      unit's code length;
//   jpeg_hscan_kernel  one workgroup per frame: exclusive scan -> bit offsets;
//   jpeg_hemit_kernel  one thread per unit: its codes MSB-first into 32-bit words
//                      at its offset (words shared with a neighbour unit by atomic
//                      OR, the rest plain stores);
//   jpeg_stuff_*       4-KB chunks: 0xFF counts, one scan over chunks and frames,
//                      then the bytes out with 0x00 after every 0xFF and the final
//                      partial byte filled with 1-bits, frames packed back to back.
namespace {

constexpr int HU_WG = 128;                               // units per workgroup (block image in LDS)
__constant__ uint8_t kZz[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                                12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                                35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                                58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

__device__ __forceinline__ int hnbits(int v) { return v ? 32 - __clz(v < 0 ? -v : v) : 0; }

struct Unit {
    int c, real;           // component; 1 = a real block, 0 = dummy
    long blk;              // block index within the frame (real)
    int dc, pred;          // this unit's DC and its predecessor's
};

// block of unit (m, c, j) of frame coefficients f: index or -1 (dummy)
__device__ __forceinline__ long unit_block(const JpegHuffArgs& a, int m, int c, int j) {
    const int hs = c ? 1 : a.hl;
    const int my = m / a.mcux, mx = m - my * a.mcux;
    const int yy = j / hs, xx = j - yy * hs;
    const int by = my * (c ? 1 : a.vl) + yy, bx = mx * hs + xx;
    return (by < a.bh[c] && bx < a.bw[c]) ? a.cblk[c] + (long)by * a.bw[c] + bx : -1;
}

// DC of unit (m, c, j): its own, or for a dummy the DC of the unit before it in the MCU (0 for the first)
__device__ __forceinline__ int unit_dc(const JpegHuffArgs& a, const int16_t* f, int m, int c, int j) {
    for (; j >= 0; --j) {
        const long b = unit_block(a, m, c, j);
        if (b >= 0) return f[b * 64];
    }
    return 0;
}

__device__ __forceinline__ Unit decode_unit(const JpegHuffArgs& a, const int16_t* f, int u) {
    const int y = a.hl * a.vl, upm = y + 2;
    const int m = u / upm, r = u - m * upm;
    Unit t;
    t.c = r < y ? 0 : r - y + 1;
    const int j = r < y ? r : 0, nbc = t.c ? 1 : y;
    t.blk = unit_block(a, m, t.c, j);
    t.real = t.blk >= 0;
    t.dc = t.real ? f[t.blk * 64] : unit_dc(a, f, m, t.c, j - 1);
    t.pred = j > 0 ? unit_dc(a, f, m, t.c, j - 1) : (m > 0 ? unit_dc(a, f, m - 1, t.c, nbc - 1) : 0);
    return t;
}

// walk the unit's symbols: put(code, size) per Huffman code + extra bits (<= 27 bits)
template <class Put>
__device__ __forceinline__ void unit_codes(const JpegHuffArgs& a, const Unit& t, const int16_t* blk, Put put) {
    const int tdc = t.c ? 1 : 0, tac = 2 + tdc;
    const int diff = t.dc - t.pred;
    int nb = hnbits(diff);
    put(((unsigned)a.code[tdc * 256 + nb] << nb) | ((unsigned)(diff < 0 ? diff - 1 : diff) & ((1u << nb) - 1)),
        a.size[tdc * 256 + nb] + nb);
    int r = 0;
    if (t.real) {
        for (int k = 1; k < 64; ++k) {
            const int v = blk[kZz[k]];
            if (v == 0) { ++r; continue; }
            for (; r > 15; r -= 16) put(a.code[tac * 256 + 0xF0], a.size[tac * 256 + 0xF0]);
            nb = hnbits(v);
            const int sym = (r << 4) + nb;
            put(((unsigned)a.code[tac * 256 + sym] << nb) | ((unsigned)(v < 0 ? v - 1 : v) & ((1u << nb) - 1)),
                a.size[tac * 256 + sym] + nb);
            r = 0;
        }
    } else {
        r = 63;
    }
    if (r) put(a.code[tac * 256], a.size[tac * 256]);
}

// the unit's 64 coefficients into LDS (zigzag reads then hit LDS, not registers)
__device__ __forceinline__ const int16_t* stage_block(const int16_t* f, const Unit& t, int16_t (*lds)[64]) {
    int16_t* d = lds[threadIdx.x];
    if (t.real) {
        const uint4* s = (const uint4*)(f + t.blk * 64);
#pragma unroll
        for (int i = 0; i < 8; ++i) ((uint4*)d)[i] = s[i];
    }
    return d;
}

__global__ __launch_bounds__(HU_WG) void jpeg_hsize_kernel(JpegHuffArgs a) {
    __shared__ __attribute__((aligned(16))) int16_t lds[HU_WG][64];
    const int fr = blockIdx.y, u = blockIdx.x * HU_WG + threadIdx.x;
    if (u >= a.units) return;
    const int16_t* f = a.coef + (size_t)fr * a.blocks_per_frame * 64;
    const Unit t = decode_unit(a, f, u);
    const int16_t* blk = stage_block(f, t, lds);
    unsigned n = 0;
    unit_codes(a, t, blk, [&](unsigned, int sz) { n += (unsigned)sz; });
    a.bits[(size_t)fr * a.units + u] = n;
}

__global__ __launch_bounds__(1024) void jpeg_hscan_kernel(JpegHuffArgs a) {
    __shared__ unsigned part[1024];
    const int fr = blockIdx.x, tid = threadIdx.x;
    unsigned* b = a.bits + (size_t)fr * a.units;
    const int per = (a.units + 1023) / 1024, lo = min(tid * per, a.units), hi = min(lo + per, a.units);
    unsigned s = 0;
    for (int i = lo; i < hi; ++i) s += b[i];
    part[tid] = s;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {                 // inclusive Hillis-Steele scan
        const unsigned v = tid >= o ? part[tid - o] : 0u;
        __syncthreads();
        part[tid] += v;
        __syncthreads();
    }
    unsigned run = part[tid] - s;                         // exclusive
    for (int i = lo; i < hi; ++i) {
        const unsigned v = b[i];
        b[i] = run;
        run += v;
    }
    if (tid == 1023) a.total[fr] = part[1023];
}

__global__ __launch_bounds__(HU_WG) void jpeg_hemit_kernel(JpegHuffArgs a) {
    __shared__ __attribute__((aligned(16))) int16_t lds[HU_WG][64];
    const int fr = blockIdx.y, u = blockIdx.x * HU_WG + threadIdx.x;
    if (u >= a.units) return;
    const int16_t* f = a.coef + (size_t)fr * a.blocks_per_frame * 64;
    const Unit t = decode_unit(a, f, u);
    const int16_t* blk = stage_block(f, t, lds);
    const unsigned off = a.bits[(size_t)fr * a.units + u];
    unsigned* w = a.words + (size_t)fr * a.wcap + (off >> 5);
    const int lead = (int)(off & 31);
    unsigned long long acc = 0;
    int n = lead;                                         // pending bits (the first `lead` belong to the neighbour)
    bool first = true;
    unit_codes(a, t, blk, [&](unsigned code, int sz) {
        acc = (acc << sz) | (code & ((1u << sz) - 1));
        n += sz;
        if (n >= 32) {
            n -= 32;
            const unsigned word = (unsigned)(acc >> n);
            if (first && lead) atomicOr(w, word);          // shared with the unit before
            else *w = word;
            first = false;
            ++w;
        }
    });
    if (n > 0) atomicOr(w, (unsigned)(acc << (32 - n)));  // shared with the unit after (or the frame's end)
}

// stuffing, over 4-KB chunks of a frame's bytes (256 threads x 16 bytes): byte i of
// frame f lands at segbase[f] + i + (0xFF bytes before i)
__device__ __forceinline__ unsigned stuff_byte(const unsigned* w, long i, long nbytes, unsigned pad) {
    unsigned v = (w[i >> 2] >> (24 - 8 * (int)(i & 3))) & 0xFFu;
    if (i == nbytes - 1) v |= (1u << pad) - 1u;        // jchuff.c flush_bits: fill with 1-bits
    return v;
}

__global__ __launch_bounds__(256) void jpeg_stuff_count_kernel(JpegHuffArgs a) {
    __shared__ unsigned red[256];
    const int fr = blockIdx.y, tid = threadIdx.x;
    const long nbytes = ((long)a.total[fr] + 7) / 8;
    const unsigned pad = (unsigned)(nbytes * 8 - a.total[fr]);
    const unsigned* w = a.words + (size_t)fr * a.wcap;
    const long b0 = (long)blockIdx.x * 4096 + tid * 16;
    unsigned ff = 0;
    for (int k = 0; k < 16; ++k)
        if (b0 + k < nbytes) ff += stuff_byte(w, b0 + k, nbytes, pad) == 0xFFu;
    red[tid] = ff;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (tid < o) red[tid] += red[tid + o];
        __syncthreads();
    }
    if (tid == 0) a.ffcnt[(size_t)fr * a.nchunk + blockIdx.x] = red[0];
}

// one workgroup: per frame the exclusive scan of its chunk counts (-> chunk output
// offsets), its stuffed length and the packed frame offsets
__global__ __launch_bounds__(1024) void jpeg_stuff_scan_kernel(JpegHuffArgs a) {
    __shared__ unsigned part[1024];
    const int tid = threadIdx.x;
    unsigned long long base = 0;
    for (int fr = 0; fr < a.n; ++fr) {
        unsigned* c = a.ffcnt + (size_t)fr * a.nchunk;
        const int per = (a.nchunk + 1023) / 1024, lo = min(tid * per, a.nchunk), hi = min(lo + per, a.nchunk);
        unsigned s = 0;
        for (int i = lo; i < hi; ++i) s += c[i];
        part[tid] = s;
        __syncthreads();
        for (int o = 1; o < 1024; o <<= 1) {
            const unsigned v = tid >= o ? part[tid - o] : 0u;
            __syncthreads();
            part[tid] += v;
            __syncthreads();
        }
        unsigned run = part[tid] - s;
        for (int i = lo; i < hi; ++i) {
            const unsigned v = c[i];
            c[i] = run;
            run += v;
        }
        const unsigned long long len = ((unsigned long long)a.total[fr] + 7) / 8 + part[1023];
        if (tid == 0) {
            a.segbase[fr] = base;
            a.segsize[fr] = len <= (unsigned long long)a.segcap ? (unsigned)len : 0xFFFFFFFFu;
        }
        base += len <= (unsigned long long)a.segcap ? len : 0ull;   // an oversize frame is not written
        __syncthreads();                                   // part[] reused by the next frame
    }
    if (tid == 0) a.segbase[a.n] = base;
}

__global__ __launch_bounds__(256) void jpeg_stuff_write_kernel(JpegHuffArgs a) {
    __shared__ unsigned part[256];
    const int fr = blockIdx.y, tid = threadIdx.x;
    if (a.segsize[fr] == 0xFFFFFFFFu) return;          // over capacity: reported, not written
    const long nbytes = ((long)a.total[fr] + 7) / 8;
    const unsigned pad = (unsigned)(nbytes * 8 - a.total[fr]);
    const unsigned* w = a.words + (size_t)fr * a.wcap;
    const long b0 = (long)blockIdx.x * 4096 + tid * 16;
    unsigned v[16], ff = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        v[k] = b0 + k < nbytes ? stuff_byte(w, b0 + k, nbytes, pad) : 0u;
        ff += (b0 + k < nbytes) & (v[k] == 0xFFu);
    }
    part[tid] = ff;
    __syncthreads();
    for (int o = 1; o < 256; o <<= 1) {
        const unsigned x = tid >= o ? part[tid - o] : 0u;
        __syncthreads();
        part[tid] += x;
        __syncthreads();
    }
    long pos = b0 + a.ffcnt[(size_t)fr * a.nchunk + blockIdx.x] + (part[tid] - ff);
    uint8_t* o = a.seg + a.segbase[fr];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        if (b0 + k >= nbytes) break;
        o[pos++] = (uint8_t)v[k];
        if (v[k] == 0xFFu) o[pos++] = 0;
    }
}

}  // namespace

hipError_t vd_launch_jpeg_huff(const JpegHuffArgs& a, hipStream_t s) {
    if (a.n <= 0 || a.units <= 0) return hipSuccess;
    hipError_t e = hipMemsetAsync(a.words, 0, (size_t)a.n * a.wcap * 4, s);
    if (e != hipSuccess) return e;
    const dim3 g((unsigned)((a.units + HU_WG - 1) / HU_WG), (unsigned)a.n);
    hipLaunchKernelGGL(jpeg_hsize_kernel, g, dim3(HU_WG), 0, s, a);
    hipLaunchKernelGGL(jpeg_hscan_kernel, dim3((unsigned)a.n), dim3(1024), 0, s, a);
    hipLaunchKernelGGL(jpeg_hemit_kernel, g, dim3(HU_WG), 0, s, a);
    return hipGetLastError();
}

hipError_t vd_launch_jpeg_stuff(const JpegHuffArgs& a, hipStream_t s) {
    if (a.n <= 0 || a.nchunk <= 0) return hipSuccess;
    const dim3 g((unsigned)a.nchunk, (unsigned)a.n);
    hipLaunchKernelGGL(jpeg_stuff_count_kernel, g, dim3(256), 0, s, a);
    hipLaunchKernelGGL(jpeg_stuff_scan_kernel, dim3(1), dim3(1024), 0, s, a);
    hipLaunchKernelGGL(jpeg_stuff_write_kernel, g, dim3(256), 0, s, a);
    return hipGetLastError();
}
