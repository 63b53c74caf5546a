// vd_math.h — arithmetic shared bit-for-bit with the CPU oracle.
//
// Every float op on the post-processing path is spelled with an explicit
// round-to-nearest intrinsic so hipcc cannot contract it into an FMA: the
// oracle (numpy float32/float64, oracle/bbox.py, oracle/vdexp.py) performs the
// same ops one rounding at a time, in the reference's order
// (detect_face/utils/utils_bbox.py:12-59,103-130).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define VD_HD __host__ __device__ __forceinline__

#if defined(__HIP_DEVICE_COMPILE__)
#define VD_FADD(a, b) __fadd_rn((a), (b))
#define VD_FSUB(a, b) __fsub_rn((a), (b))
#define VD_FMUL(a, b) __fmul_rn((a), (b))
#define VD_FDIV(a, b) __fdiv_rn((a), (b))
#define VD_DADD(a, b) __dadd_rn((a), (b))
#define VD_DSUB(a, b) __dsub_rn((a), (b))
#define VD_DMUL(a, b) __dmul_rn((a), (b))
#else
// host side is compiled with -ffp-contract=off (see build.py)
#define VD_FADD(a, b) ((float)(a) + (float)(b))
#define VD_FSUB(a, b) ((float)(a) - (float)(b))
#define VD_FMUL(a, b) ((float)(a) * (float)(b))
#define VD_FDIV(a, b) ((float)(a) / (float)(b))
#define VD_DADD(a, b) ((double)(a) + (double)(b))
#define VD_DSUB(a, b) ((double)(a) - (double)(b))
#define VD_DMUL(a, b) ((double)(a) * (double)(b))
#endif

VD_HD double vd_bits_to_double(uint64_t u) { return __builtin_bit_cast(double, u); }

// Deterministic float32 exp: widen to double, Cody-Waite reduction with
// LN2_HI having 21 trailing zero bits (n*LN2_HI exact), degree-13 Taylor
// Horner in plain double ops, exact 2^n scaling, one final rounding to float.
// Twin of oracle/vdexp.py:vd_expf (same constants, same op order).
VD_HD float vd_expf(float xf) {
    double x = (double)xf;
    if (x != x) return xf;                     // NaN
    if (x > 89.0) return __builtin_huge_valf();
    if (x < -104.0) return 0.0f;
    const double LOG2E = vd_bits_to_double(0x3ff71547652b82feULL);
    const double LN2_HI = vd_bits_to_double(0x3fe62e42fee00000ULL);
    const double LN2_LO = vd_bits_to_double(0x3dea39ef35793c76ULL);
    double n = __builtin_rint(VD_DMUL(x, LOG2E));   // round half to even, like np.rint
    double r = VD_DSUB(VD_DSUB(x, VD_DMUL(n, LN2_HI)), VD_DMUL(n, LN2_LO));
    double p = vd_bits_to_double(0x3de6124613a86d09ULL);   // 1/13!
    p = VD_DADD(VD_DMUL(p, r), vd_bits_to_double(0x3e21eed8eff8d898ULL));  // 1/12!
    p = VD_DADD(VD_DMUL(p, r), vd_bits_to_double(0x3e5ae64567f544e4ULL));  // 1/11!
    p = VD_DADD(VD_DMUL(p, r), vd_bits_to_double(0x3e927e4fb7789f5cULL));  // 1/10!
    p = VD_DADD(VD_DMUL(p, r), vd_bits_to_double(0x3ec71de3a556c734ULL));  // 1/9!
    p = VD_DADD(VD_DMUL(p, r), vd_bits_to_double(0x3efa01a01a01a01aULL));  // 1/8!
    p = VD_DADD(VD_DMUL(p, r), vd_bits_to_double(0x3f2a01a01a01a01aULL));  // 1/7!
    p = VD_DADD(VD_DMUL(p, r), vd_bits_to_double(0x3f56c16c16c16c17ULL));  // 1/6!
    p = VD_DADD(VD_DMUL(p, r), vd_bits_to_double(0x3f81111111111111ULL));  // 1/5!
    p = VD_DADD(VD_DMUL(p, r), vd_bits_to_double(0x3fa5555555555555ULL));  // 1/4!
    p = VD_DADD(VD_DMUL(p, r), vd_bits_to_double(0x3fc5555555555555ULL));  // 1/3!
    p = VD_DADD(VD_DMUL(p, r), 0.5);
    p = VD_DADD(VD_DMUL(p, r), 1.0);
    p = VD_DADD(VD_DMUL(p, r), 1.0);
    // exact scaling by 2^n (|n| <= 151; split so each factor is a normal double)
    int ni = (int)n;
    int n1 = ni / 2, n2 = ni - n1;
    double s1 = __builtin_bit_cast(double, (uint64_t)(int64_t)(n1 + 1023) << 52);
    double s2 = __builtin_bit_cast(double, (uint64_t)(int64_t)(n2 + 1023) << 52);
    return (float)VD_DMUL(VD_DMUL(p, s1), s2);
}

// torchvision nms IoU test (nms_kernel.cpp [ext]): float32 ops, double compare.
VD_HD bool vd_iou_gt(float ix1, float iy1, float ix2, float iy2, float iarea,
                     float jx1, float jy1, float jx2, float jy2, float jarea, double thr) {
    float xx1 = ix1 > jx1 ? ix1 : jx1;
    float yy1 = iy1 > jy1 ? iy1 : jy1;
    float xx2 = ix2 < jx2 ? ix2 : jx2;
    float yy2 = iy2 < jy2 ? iy2 : jy2;
    float w = VD_FSUB(xx2, xx1);
    float h = VD_FSUB(yy2, yy1);
    w = w > 0.0f ? w : 0.0f;
    h = h > 0.0f ? h : 0.0f;
    float inter = VD_FMUL(w, h);
    float ovr = VD_FDIV(inter, VD_FSUB(VD_FADD(iarea, jarea), inter));
    return (double)ovr > thr;
}
