// dwconv.hip — depthwise 3x3 conv + BatchNorm(eval) + activation, NHWC.
//
// The conv_dw blocks of the MobileNetV1-0.25 RetinaFace backbone
// (detect_face/nets/mobilenet025.py:10-19: Conv2d(inp, inp, 3, stride, 1,
// groups=inp) + BatchNorm2d + LeakyReLU(0.1)), selected by the reference's
// `backbone="mobilenet"` option (face.py:35, retinaface.py:60-61). One output
// channel reads one input channel, so the layer is pure HBM traffic (9 taps of 16 B
// per 8 channels, mostly L2 hits, one 16-B store): one thread per (pixel, 16-B
// channel vector), f32 accumulation over the taps in (dy, dx) order, the same
// acc*scale + shift + activation epilogue as the dense convs.
#include "vd_common.h"

namespace {

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

template <typename T> struct DwVec;
template <> struct DwVec<__bf16> { static constexpr int N = 8; };
template <> struct DwVec<_Float16> { static constexpr int N = 8; };
template <> struct DwVec<float>  { static constexpr int N = 4; };

__device__ __forceinline__ float act_apply(float v, int act, float slope) {
    if (act == VD_ACT_RELU) return v > 0.f ? v : 0.f;
    if (act == VD_ACT_LEAKY) return v > 0.f ? v : v * slope;
    if (act == VD_ACT_SILU) return v / (1.0f + __expf(-v));
    return v;
}

template <typename T>
__global__ __launch_bounds__(256) void dwconv3x3_kernel(DwConvArgs a) {
    constexpr int N = DwVec<T>::N;
    const int cv = a.c / N;
    const long idx = (long)blockIdx.x * 256 + threadIdx.x;
    const long total = (long)a.B * a.yh * a.yw * cv;
    const bool valid = idx < total;          // no early exit: the wave merges its output max
    const long ic = valid ? idx : total - 1;
    const int g = (int)(ic % cv);
    long pix = ic / cv;
    const int ox = (int)(pix % a.yw);
    pix /= a.yw;
    const int oy = (int)(pix % a.yh);
    const int b = (int)(pix / a.yh);
    const int c0 = g * N;
    float acc[N];
#pragma unroll
    for (int e = 0; e < N; ++e) acc[e] = 0.f;
    const T* x = (const T*)a.x;
    const T* w = (const T*)a.w;
#pragma unroll
    for (int dy = 0; dy < 3; ++dy) {
        const int iy = oy * a.stride - 1 + dy;
        if ((unsigned)iy >= (unsigned)a.xh) continue;
#pragma unroll
        for (int dx = 0; dx < 3; ++dx) {
            const int ix = ox * a.stride - 1 + dx;
            if ((unsigned)ix >= (unsigned)a.xw) continue;
            const u32x4 xv = *(const u32x4*)(x + (((size_t)b * a.xh + iy) * a.xw + ix) * a.ldx + a.xcoff + c0);
            const u32x4 wv = *(const u32x4*)(w + (size_t)(dy * 3 + dx) * a.c + c0);
            const T* xe = (const T*)&xv;
            const T* we = (const T*)&wv;
#pragma unroll
            for (int e = 0; e < N; ++e) acc[e] += (float)xe[e] * (float)we[e];
        }
    }
    T o[N];
    float vmax = 0.f;
#pragma unroll
    for (int e = 0; e < N; ++e) {
        const float v = act_apply(acc[e] * a.scale[c0 + e] + a.shift[c0 + e], a.act, a.slope);
        o[e] = (T)v;
        vmax = fmaxf(vmax, fabsf(v));
    }
    if (a.ymax) {
        AmaxTrack t;
        if (valid) t.add(a.ymax, b, vmax);
        t.publish(a.ymax);
    }
    if (valid) *(u32x4*)((T*)a.y + (((size_t)b * a.yh + oy) * a.yw + ox) * a.ldy + a.ycoff + c0) = *(const u32x4*)o;
}

}  // namespace

hipError_t vd_launch_dwconv(const DwConvArgs& a, bool f32, bool f16, hipStream_t s) {
    const int n = f32 ? 4 : 8;
    if (a.c % n || a.ldx % n || a.xcoff % n || a.ldy % n || a.ycoff % n) return hipErrorInvalidValue;
    const long total = (long)a.B * a.yh * a.yw * (a.c / n);
    if (total <= 0) return hipSuccess;
    const dim3 grid((unsigned)((total + 255) / 256));
    if (f32) hipLaunchKernelGGL(dwconv3x3_kernel<float>, grid, dim3(256), 0, s, a);
    else if (f16) hipLaunchKernelGGL(dwconv3x3_kernel<_Float16>, grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL(dwconv3x3_kernel<__bf16>, grid, dim3(256), 0, s, a);
    return hipGetLastError();
}
