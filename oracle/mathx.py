"""Deterministic exp / log / standard-normal draws, restating
uptune_amd/csrc/ut_core.h operation for operation (numpy float64 elementwise
ops are single IEEE operations, so the bits agree with the device build
compiled with -ffp-contract=off).

These replace `random.gauss` / `random.normalvariate` (CPython Lib/random.py)
and `numpy.exp` in the PSO sigmoid (manipulator.py:694, 992) for the
counter-based RNG; libm results could differ from the device by an ulp.
"""
import numpy as np

from . import philox as ph

LN2_HI = 6.93147180369123816490e-01
LN2_LO = 1.90821492927058770002e-10
INV_LN2 = 1.44269504088896338700e+00
SQRT2 = 1.41421356237309514547e+00

_LOG_C = [1.0 / k for k in (23, 21, 19, 17, 15, 13, 11, 9, 7, 5, 3)]
_EXP_C = [1.0 / 6227020800.0, 1.0 / 479001600.0, 1.0 / 39916800.0, 1.0 / 3628800.0, 1.0 / 362880.0,
          1.0 / 40320.0, 1.0 / 5040.0, 1.0 / 720.0, 1.0 / 120.0, 1.0 / 24.0, 1.0 / 6.0, 0.5, 1.0, 1.0]


def ut_log(x):
    x = np.asarray(x, dtype=np.float64)
    b = x.view(np.uint64)
    e = ((b >> np.uint64(52)) & np.uint64(0x7FF)).astype(np.int64) - 1023
    frac = b & np.uint64(0x000FFFFFFFFFFFFF)
    m = (frac | np.uint64(0x3FF0000000000000)).view(np.float64)
    big = m > SQRT2
    m = np.where(big, (frac | np.uint64(0x3FE0000000000000)).view(np.float64), m)
    e = e + big.astype(np.int64)
    s = (m - 1.0) / (m + 1.0)
    s2 = s * s
    p = np.full_like(s, _LOG_C[0])
    for c in _LOG_C[1:]:
        p = p * s2 + c
    lm = (2.0 * s) + ((2.0 * s) * (s2 * p))
    fe = e.astype(np.float64)
    return (fe * LN2_HI) + ((fe * LN2_LO) + lm)


def ut_exp(x):
    x = np.asarray(x, dtype=np.float64)
    kd = np.rint(x * INV_LN2)
    r = (x - kd * LN2_HI) - kd * LN2_LO
    p = np.full_like(r, _EXP_C[0])
    for c in _EXP_C[1:]:
        p = p * r + c
    k = np.clip(kd, -2000, 2000).astype(np.int64)
    hi = k > 1023
    p = np.where(hi, p * 2.0, p)
    k = np.where(hi, k - 1, k)
    lo = k < -1021
    with np.errstate(over="ignore", under="ignore"):
        k_norm = np.clip(np.where(lo, 0, k), -1022, 1023)
        out = p * ((k_norm + 1023).astype(np.uint64) << np.uint64(52)).view(np.float64)
        k_sub = np.where(lo, k + 1000, 0)
        two_m1000 = np.array([(-1000 + 1023) << 52], dtype=np.uint64).view(np.float64)[0]
        sub = (p * ((k_sub + 1023).astype(np.uint64) << np.uint64(52)).view(np.float64)) * two_m1000
    out = np.where(lo, sub, out)
    out = np.where(x > 709.782712893384, np.inf, out)
    out = np.where(x < -745.2, 0.0, out)
    out = np.where(np.isnan(x), x, out)
    return out


def normal_draw(seed, cand, stream, round_, op):
    """vectorised over cand (uint64 array); same attempt order as the device"""
    cand = np.asarray(cand, dtype=np.uint64)
    out = np.zeros(cand.shape, dtype=np.float64)
    done = np.zeros(cand.shape, dtype=bool)
    for a in range(16):
        x, y, z, w = ph.draw(seed, cand, (int(stream) | (a << 24)) & 0xFFFFFFFF, round_, op)
        u = 2.0 * ph.u01(x, y) - 1.0
        v = 2.0 * ph.u01(z, w) - 1.0
        s = u * u + v * v
        ok = (s > 0.0) & (s < 1.0) & ~done
        if ok.any():
            ss = s[ok]
            out[ok] = u[ok] * np.sqrt((-2.0 * ut_log(ss)) / ss)
            done |= ok
        if done.all():
            break
    return out
