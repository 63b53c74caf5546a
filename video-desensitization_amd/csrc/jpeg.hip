// jpeg.hip — device stage of the JPEG frame decode (host stage: jpeg_host.cpp).
//
// libjpeg-turbo's default decode path [ext], as cv2.imread runs it on the
// reference's ffmpeg-split frames (combine_detect.py:167-172), restated
// bit-exactly (oracle/jpeg.py, pinned against Pillow's libjpeg-turbo):
//   jpeg_idct_kernel   8 lanes per 8x8 block: scatter the block's sparse
//                      coefficients dequantized into LDS, jidctint.c ISLOW column
//                      pass (lane = column), row pass (lane = row) with the
//                      post-IDCT range_limit table, 8 samples per 8-B store into
//                      the component plane (block-major: 64 B per block);
//   jpeg_color_kernel  one lane per output pixel: jdsample.c fancy upsampling
//                      (h2v1 / h2v2 triangle filters, edge rows/columns
//                      replicated) of the chroma planes and jdcolor.c
//                      ycc_rgb_convert (16-bit fixed-point tables), RGB bytes
//                      straight into the frame batch vd_process consumes.
#include "vd_common.h"

namespace {

constexpr int CONST_BITS = 13, PASS1_BITS = 2;
constexpr int F_0_298631336 = 2446, F_0_390180644 = 3196, F_0_541196100 = 4433, F_0_765366865 = 6270,
              F_0_899976223 = 7373, F_1_175875602 = 9633, F_1_501321110 = 12299, F_1_847759065 = 15137,
              F_1_961570560 = 16069, F_2_053119869 = 16819, F_2_562915447 = 20995, F_3_072711026 = 25172;

// one 1-D ISLOW pass on inputs z[0..7] (index = frequency), outputs o[0..7] (undescaled)
// (64-bit like libjpeg's JLONG, so corrupt coefficients wrap exactly as there)
typedef long long jl;
__device__ __forceinline__ void idct_1d(const jl* z, jl* o) {
    jl zz = (z[2] + z[6]) * F_0_541196100;
    const jl tmp2 = zz + z[6] * (-F_1_847759065);
    const jl tmp3 = zz + z[2] * F_0_765366865;
    const jl tmp0 = (z[0] + z[4]) * (1 << CONST_BITS);
    const jl tmp1 = (z[0] - z[4]) * (1 << CONST_BITS);
    const jl tmp10 = tmp0 + tmp3, tmp13 = tmp0 - tmp3, tmp11 = tmp1 + tmp2, tmp12 = tmp1 - tmp2;
    jl t0 = z[7], t1 = z[5], t2 = z[3], t3 = z[1];
    jl z1 = t0 + t3, z2 = t1 + t2, z3 = t0 + t2, z4 = t1 + t3;
    const jl z5 = (z3 + z4) * F_1_175875602;
    t0 *= F_0_298631336;
    t1 *= F_2_053119869;
    t2 *= F_3_072711026;
    t3 *= F_1_501321110;
    z1 *= -F_0_899976223;
    z2 *= -F_2_562915447;
    z3 = z3 * (-F_1_961570560) + z5;
    z4 = z4 * (-F_0_390180644) + z5;
    t0 += z1 + z3;
    t1 += z2 + z4;
    t2 += z2 + z3;
    t3 += z1 + z4;
    o[0] = tmp10 + t3; o[7] = tmp10 - t3;
    o[1] = tmp11 + t2; o[6] = tmp11 - t2;
    o[2] = tmp12 + t1; o[5] = tmp12 - t1;
    o[3] = tmp13 + t0; o[4] = tmp13 - t0;
}

// post-IDCT range_limit[x & RANGE_MASK] (jdmaster.c prepare_range_limit_table)
__device__ __forceinline__ unsigned range_limit_idct(jl x) {
    const int j = (int)(x & 1023);
    return j < 128 ? (unsigned)(j + 128) : (j < 512 ? 255u : (j < 896 ? 0u : (unsigned)(j - 896)));
}

constexpr int BLK_PER_WG = 32;

__global__ __launch_bounds__(256) void jpeg_idct_kernel(JpegArgs a) {
    __shared__ int coef[BLK_PER_WG][64];
    __shared__ int ws[BLK_PER_WG][64];
    const int tid = threadIdx.x, g = tid >> 3, t = tid & 7;
    const long gb = (long)blockIdx.x * BLK_PER_WG + g;
    const long total = (long)a.n * a.blocks_per_image;
    const bool live = gb < total;
#pragma unroll
    for (int k = 0; k < 8; ++k) coef[g][t * 8 + k] = 0;
    __syncthreads();
    int img = 0, lb = 0, c = 0;
    if (live) {
        img = (int)(gb / a.blocks_per_image);
        lb = (int)(gb - (long)img * a.blocks_per_image);
        c = (a.nc > 2 && lb >= a.cblk[2]) ? 2 : ((a.nc > 1 && lb >= a.cblk[1]) ? 1 : 0);
        const uint16_t* q = a.quant + ((size_t)img * 3 + c) * 64;
        if (a.dense) {
#pragma unroll
            for (int k = t * 8; k < t * 8 + 8; ++k) coef[g][k] = (int)a.dense[gb * 64 + k] * (int)q[k];
        } else {
            for (uint32_t e = a.blk_off[gb] + t; e < a.blk_off[gb + 1]; e += 8) {
                const uint32_t v = a.entries[e];
                const int k = (int)(v >> 16) & 63;
                coef[g][k] = (int)(int16_t)(v & 0xFFFFu) * (int)q[k];
            }
        }
    }
    __syncthreads();
    {   // pass 1: column t, results scaled by 2^PASS1_BITS
        jl z[8], o[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) z[u] = coef[g][u * 8 + t];
        idct_1d(z, o);
        constexpr int sh = CONST_BITS - PASS1_BITS;
#pragma unroll
        for (int u = 0; u < 8; ++u) ws[g][u * 8 + t] = (int)((o[u] + (1 << (sh - 1))) >> sh);
    }
    __syncthreads();
    if (!live) return;
    {   // pass 2: row t; the descale rounding is folded into the DC term (jidctint.c)
        jl z[8], o[8];
#pragma unroll
        for (int v = 0; v < 8; ++v) z[v] = ws[g][t * 8 + v];
        z[0] += 1 << (PASS1_BITS + 2);
        idct_1d(z, o);
        constexpr int sh = CONST_BITS + PASS1_BITS + 3;
        unsigned lo = 0, hi = 0;
#pragma unroll
        for (int v = 0; v < 4; ++v) {
            lo |= range_limit_idct(o[v] >> sh) << (8 * v);
            hi |= range_limit_idct(o[v + 4] >> sh) << (8 * v);
        }
        uint8_t* dst = a.planes + (size_t)gb * 64 + t * 8;
        *(uint2*)dst = make_uint2(lo, hi);
    }
}

// sample (x, y) of component c of image img from the block-major plane
__device__ __forceinline__ int samp(const JpegArgs& a, int img, int c, int x, int y) {
    const size_t blk = (size_t)img * a.blocks_per_image + a.cblk[c] + (size_t)(y >> 3) * a.bw[c] + (x >> 3);
    return a.planes[blk * 64 + (y & 7) * 8 + (x & 7)];
}

// jdsample.c fancy upsampling of component c at output pixel (x, y)
__device__ __forceinline__ int upsampled(const JpegArgs& a, int img, int c, int x, int y) {
    const int fx = a.fx[c], fy = a.fy[c];
    if (fx == 1 && fy == 1) return samp(a, img, c, x, y);
    const int dw = a.dw[c];                                   // downsampled_width
    const int dh = a.dh[c];                                   // downsampled_height
    const int i = x >> 1;
    if (fy == 1) {                                            // h2v1
        const int r = y, p = samp(a, img, c, i, r);
        if ((x & 1) == 0) return i == 0 ? p : (p * 3 + samp(a, img, c, i - 1, r) + 1) >> 2;
        return i == dw - 1 ? p : (p * 3 + samp(a, img, c, i + 1, r) + 2) >> 2;
    }
    // h2v2: v = 0 -> the row above is the further one, v = 1 -> the row below
    const int r = y >> 1;
    const int rr = (y & 1) == 0 ? max(r - 1, 0) : min(r + 1, dh - 1);
    auto colsum = [&](int j) { return samp(a, img, c, j, r) * 3 + samp(a, img, c, j, rr); };
    const int th = colsum(i);
    if ((x & 1) == 0) return i == 0 ? (th * 4 + 8) >> 4 : (th * 3 + colsum(i - 1) + 8) >> 4;
    return i == dw - 1 ? (th * 4 + 7) >> 4 : (th * 3 + colsum(i + 1) + 7) >> 4;
}

__device__ __forceinline__ int clamp255(int v) { return v < 0 ? 0 : (v > 255 ? 255 : v); }

__device__ __forceinline__ void pixel_rgb(const JpegArgs& a, int img, int x, int y, int& r, int& g, int& b) {
    const int Y = upsampled(a, img, 0, x, y);
    if (a.nc == 1) { r = g = b = Y; return; }
    // jdcolor.c build_ycc_rgb_table: SCALEBITS 16, FIX(x) = x * 65536 + 0.5
    const int cb = upsampled(a, img, 1, x, y) - 128, cr = upsampled(a, img, 2, x, y) - 128;
    const int cr_r = (91881 * cr + 32768) >> 16;
    const int cb_b = (116130 * cb + 32768) >> 16;
    const int gg = ((-22554 * cb + 32768) + (-46802 * cr)) >> 16;
    r = clamp255(Y + cr_r);
    g = clamp255(Y + gg);
    b = clamp255(Y + cb_b);
}

// one lane per output pixel (any width / pitch)
__global__ __launch_bounds__(256) void jpeg_color_kernel(JpegArgs a) {
    const long p = (long)blockIdx.x * 256 + threadIdx.x;
    const int img = blockIdx.y;
    if (p >= (long)a.h * a.w) return;
    const int y = (int)(p / a.w), x = (int)(p - (long)y * a.w);
    uint8_t* dst = a.out + (size_t)img * a.h * a.pitch + (size_t)y * a.pitch + (size_t)x * 3;
    int r, g, b;
    pixel_rgb(a, img, x, y, r, g, b);
    dst[0] = (uint8_t)r;
    dst[1] = (uint8_t)g;
    dst[2] = (uint8_t)b;
}

// one lane per 4 pixels of a row (w % 4 == 0, pitch % 4 == 0): 12 bytes as three
// dword stores instead of 12 byte stores, neighbouring samples shared through L1
__global__ __launch_bounds__(256) void jpeg_color4_kernel(JpegArgs a) {
    const int q = blockIdx.x * 256 + threadIdx.x;            // 4-pixel group within the image
    const int img = blockIdx.y;
    const int gw = a.w >> 2;
    if (q >= a.h * gw) return;
    const int y = q / gw, x = (q - y * gw) * 4;
    unsigned v[3] = {0u, 0u, 0u};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        int r, g, b;
        pixel_rgb(a, img, x + k, y, r, g, b);
        const int o = 3 * k;
        v[o >> 2] |= (unsigned)r << (8 * (o & 3));
        v[(o + 1) >> 2] |= (unsigned)g << (8 * ((o + 1) & 3));
        v[(o + 2) >> 2] |= (unsigned)b << (8 * ((o + 2) & 3));
    }
    unsigned* dst = (unsigned*)(a.out + (size_t)img * a.h * a.pitch + (size_t)y * a.pitch + (size_t)x * 3);
    dst[0] = v[0];
    dst[1] = v[1];
    dst[2] = v[2];
}

}  // namespace

hipError_t vd_launch_jpeg(const JpegArgs& a0, hipStream_t s) {
    JpegArgs a = a0;
    for (int c = 0; c < 3; ++c) {
        const int hs = a.hs[c] > 0 ? a.hs[c] : 1, vs = a.vs[c] > 0 ? a.vs[c] : 1;
        a.fx[c] = a.hmax / hs;
        a.fy[c] = a.vmax / vs;
        a.dw[c] = (a.w * hs + a.hmax - 1) / a.hmax;
        a.dh[c] = (a.h * vs + a.vmax - 1) / a.vmax;
    }
    const long total = (long)a.n * a.blocks_per_image;
    if (total <= 0) return hipSuccess;
    hipLaunchKernelGGL(jpeg_idct_kernel, dim3((unsigned)((total + BLK_PER_WG - 1) / BLK_PER_WG)), dim3(256), 0, s, a);
    const long px = (long)a.h * a.w;
    if ((a.w & 3) == 0 && (a.pitch & 3) == 0 && ((uintptr_t)a.out & 3) == 0 && px / 4 < (1L << 31))
        hipLaunchKernelGGL(jpeg_color4_kernel, dim3((unsigned)((px / 4 + 255) / 256), a.n), dim3(256), 0, s, a);
    else
        hipLaunchKernelGGL(jpeg_color_kernel, dim3((unsigned)((px + 255) / 256), a.n), dim3(256), 0, s, a);
    return hipGetLastError();
}
