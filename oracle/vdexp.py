"""Deterministic float32 exp shared bit-for-bit by the oracle and the HIP kernels.

The reference evaluates ``torch.exp`` (decode, utils_bbox.py:51) and the softmax
``exp`` (retinaface.py:147) inside torch's vectorised kernels [ext]; those are
not reproducible bit-for-bit off their own library. Both sides of the parity
check therefore use one fully specified function: the float32 input is widened
to double, ``exp`` is evaluated with plain IEEE double operations (no FMA,
every op correctly rounded, so numpy and the GPU ``__d*_rn`` intrinsics agree
exactly), and the result is rounded to float32 once. Its error against the
true exp is below 1e-15 relative before the final rounding, i.e. it is the
correctly rounded expf except within ~1e-15 of a rounding boundary -- at least
as close to the truth as torch's 1-ulp SLEEF/CUDA expf. The device twin is
``vd_expf`` in video-desensitization_amd/csrc/vd_math.h.
Test infrastructure only.
"""
import numpy as np

LOG2E = 1.4426950408889634            # 0x3FF71547652B82FE
LN2_HI = 6.93147180369123816490e-01   # 0x3FE62E42FEE00000: low 21 bits zero -> n*LN2_HI exact
LN2_LO = 1.90821492927058770002e-10   # 0x3DEA39EF35793C76
# Taylor coefficients 1/k!, k = 13..0 (Horner, |r| <= 0.3466)
COEF = [1.0 / 6227020800.0, 1.0 / 479001600.0, 1.0 / 39916800.0, 1.0 / 3628800.0,
        1.0 / 362880.0, 1.0 / 40320.0, 1.0 / 5040.0, 1.0 / 720.0, 1.0 / 120.0,
        1.0 / 24.0, 1.0 / 6.0, 0.5, 1.0, 1.0]
HI_CUT = 89.0      # exp(89) > FLT_MAX -> +inf after rounding
LO_CUT = -104.0    # exp(-104) < FLT_TRUE_MIN/2 -> +0 after rounding


def vd_expf(x):
    """x: float32 array (or scalar) -> float32 array."""
    x = np.asarray(x, dtype=np.float32)
    xd = x.astype(np.float64)
    xc = np.clip(xd, LO_CUT, HI_CUT)
    n = np.rint(xc * LOG2E)
    r = (xc - n * LN2_HI) - n * LN2_LO
    p = np.full_like(r, COEF[0])
    for c in COEF[1:]:
        p = p * r + c
    y = np.ldexp(p, n.astype(np.int64))
    y = np.where(xd > HI_CUT, np.inf, y)
    y = np.where(xd < LO_CUT, 0.0, y)
    y = np.where(np.isnan(xd), np.nan, y)
    return y.astype(np.float32)
