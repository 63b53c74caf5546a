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
