"""Philox4x32-10 counter RNG (Salmon et al. SC'11), vectorised over numpy
uint32 arrays; the same counter layout as uptune_amd/csrc/ut_core.h:

    counter = (cand_lo, cand_hi, stream, (round << 8) | op),  key = (seed_lo, seed_hi)

This replaces the reference's single MT19937 stream (python `random`),
whose draw order is data dependent.
"""
import numpy as np

M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
W0, W1 = 0x9E3779B9, 0xBB67AE85
MASK32 = np.uint64(0xFFFFFFFF)

OP_INIT, OP_DE, OP_PSO, OP_GA, OP_GGA = 1, 2, 3, 4, 5
STREAM_CAND = 0xFFFF0000
STREAM_RETRY_SHIFT = 20
STREAM_SUB_SHIFT = 28


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    c0, c1, c2, c3 = (np.asarray(x, dtype=np.uint64) & MASK32 for x in (c0, c1, c2, c3))
    c0, c1, c2, c3 = np.broadcast_arrays(c0, c1, c2, c3)
    k0, k1 = int(k0) & 0xFFFFFFFF, int(k1) & 0xFFFFFFFF
    for _ in range(10):
        p0 = M0 * c0
        p1 = M1 * c2
        hi0, lo0 = p0 >> np.uint64(32), p0 & MASK32
        hi1, lo1 = p1 >> np.uint64(32), p1 & MASK32
        c0, c1, c2, c3 = hi1 ^ c1 ^ np.uint64(k0), lo1, hi0 ^ c3 ^ np.uint64(k1), lo0
        k0 = (k0 + W0) & 0xFFFFFFFF
        k1 = (k1 + W1) & 0xFFFFFFFF
    return c0, c1, c2, c3


def draw(seed, cand, stream, round_, op):
    cand = np.asarray(cand, dtype=np.uint64)
    return philox4x32_10(cand & MASK32, cand >> np.uint64(32), np.uint64(stream),
                         np.uint64(((int(round_) << 8) | int(op)) & 0xFFFFFFFF),
                         int(seed) & 0xFFFFFFFF, (int(seed) >> 32) & 0xFFFFFFFF)


def u01(lo, hi):
    """53-bit uniform in [0, 1)"""
    v = ((np.asarray(hi, dtype=np.uint64) << np.uint64(32)) | np.asarray(lo, dtype=np.uint64)) >> np.uint64(11)
    return v.astype(np.float64) * (1.0 / 9007199254740992.0)


def u64(lo, hi):
    return (np.asarray(hi, dtype=np.uint64) << np.uint64(32)) | np.asarray(lo, dtype=np.uint64)


def mulhi64(a, b):
    a = np.asarray(a, dtype=np.uint64)
    b = np.asarray(b, dtype=np.uint64)
    a_lo, a_hi = a & MASK32, a >> np.uint64(32)
    b_lo, b_hi = b & MASK32, b >> np.uint64(32)
    ll = a_lo * b_lo
    hl = a_hi * b_lo
    lh = a_lo * b_hi
    hh = a_hi * b_hi
    cross = (ll >> np.uint64(32)) + (hl & MASK32) + lh
    return hh + (hl >> np.uint64(32)) + (cross >> np.uint64(32))


def below64(x, n):
    """floor(x * n / 2^64): integer in [0, n)"""
    return mulhi64(x, np.uint64(n))


def umulhi32(w, n):
    return (np.asarray(w, dtype=np.uint64) * np.uint64(n)) >> np.uint64(32)
