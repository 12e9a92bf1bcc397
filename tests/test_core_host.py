"""The shared device arithmetic (uptune_amd/csrc/ut_core.h), compiled for the
host with g++, against CPython's repr / hashlib and the oracle's Philox.
This exercises the exact source the gfx950 kernels compile (CPU, no GPU)."""
import ctypes
import hashlib
import math
import os
import random
import struct
import subprocess

import numpy as np
import pytest

from oracle import philox as ph

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HOSTLIB = os.path.join(ROOT, "uptune_amd", "libuthot_hostcheck.so")


@pytest.fixture(scope="module")
def hc():
    src = os.path.join(ROOT, "uptune_amd", "csrc", "hostcheck.cpp")
    if not os.path.exists(HOSTLIB) or os.path.getmtime(HOSTLIB) < os.path.getmtime(src):
        subprocess.check_call(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-ffp-contract=off", src, "-o",
                               HOSTLIB])
    lib = ctypes.CDLL(HOSTLIB)
    lib.uthc_repr_double.argtypes = [ctypes.c_double, ctypes.c_char_p]
    lib.uthc_repr_int64.argtypes = [ctypes.c_longlong, ctypes.c_char_p]
    lib.uthc_sha256.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p]
    lib.uthc_philox.argtypes = [ctypes.c_ulonglong, ctypes.c_ulonglong, ctypes.c_uint, ctypes.c_uint, ctypes.c_uint,
                                ctypes.POINTER(ctypes.c_uint)]
    return lib


def _repr(lib, x):
    buf = ctypes.create_string_buffer(64)
    n = lib.uthc_repr_double(x, buf)
    return buf.raw[:n].decode()


SPECIAL = [0.0, -0.0, 1.0, -1.0, 0.1, 0.2, 0.3, 1e16, 1e15, 9999999999999998.0, 1e-4, 1e-5, 0.00012345,
           123.456, 5e-324, -5e-324, 2.2250738585072014e-308, 2.225073858507201e-308, 1.7976931348623157e308,
           float("inf"), float("-inf"), 9007199254740993.0, 1e22, 1e23, 2.0 ** 63, 2.0 ** -1074 * 3, 1 / 3,
           -1000.0, 1000.0, 999.9999999999999, 4.35, 2.675, 1e300, 1e-300, 100.0, 12345678901234567890.0]


def test_repr_special(hc):
    for x in SPECIAL:
        assert _repr(hc, x) == repr(x), x
    assert _repr(hc, float("nan")) == "nan"


def test_repr_random_bits(hc):
    rng = random.Random(12345)
    for _ in range(200000):
        x = struct.unpack("<d", struct.pack("<Q", rng.getrandbits(64)))[0]
        if math.isnan(x):
            continue
        assert _repr(hc, x) == repr(x)


def test_repr_search_ranges(hc):
    rng = random.Random(99)
    for lo, hi in [(-1000.0, 1000.0), (0.0, 1.0), (-1e-3, 1e-3), (1e10, 1e18)]:
        for _ in range(50000):
            x = rng.uniform(lo, hi)
            assert _repr(hc, x) == repr(x)
    # values produced by set_unit_value arithmetic: u * span + lo
    for _ in range(50000):
        u = rng.random()
        x = u * 2000.0 + -1000.0
        assert _repr(hc, x) == repr(x)


def test_repr_integral_floats(hc):
    """integers in [1, 2^53) take the small-integer path of repr_double"""
    rng = random.Random(7)
    xs = [float(v) for v in range(1, 20001)] + [float(10 ** k) for k in range(16)]
    xs += [float(2 ** k) for k in range(54)] + [float(2 ** 53 - 1), float(2 ** 53), float(2 ** 53 + 2)]
    xs += [float(rng.randrange(1, 2 ** 53)) for _ in range(20000)]
    xs += [float(rng.randrange(1, 10 ** 6) * 10 ** rng.randrange(0, 10)) for _ in range(20000)]
    xs += [math.nextafter(x, 0.0) for x in xs[:3000]] + [math.nextafter(x, math.inf) for x in xs[:3000]]
    for x in xs:
        assert _repr(hc, x) == repr(x), x
        assert _repr(hc, -x) == repr(-x), -x


def test_repr_int(hc):
    buf = ctypes.create_string_buffer(32)
    for v in [0, 1, -1, 9, 10, 99, 100, 2**31, -2**31, 2**53 + 1, 2**63 - 1, -2**63, 107572959]:
        n = hc.uthc_repr_int64(v, buf)
        assert buf.raw[:n].decode() == repr(v)


def test_sha256(hc):
    rng = random.Random(3)
    out = ctypes.create_string_buffer(32)
    for L in [0, 1, 3, 55, 56, 63, 64, 65, 119, 120, 127, 128, 4588, 30178]:
        m = bytes(rng.getrandbits(8) for _ in range(L))
        hc.uthc_sha256(m, L, out)
        assert out.raw == hashlib.sha256(m).digest()


def test_philox_matches_oracle(hc):
    out = (ctypes.c_uint * 4)()
    for seed, cand, stream, rnd, op in [(0, 0, 0, 0, 1), (2**40 + 7, 123456789, 5, 17, 2),
                                        (1, 2**33 + 5, 0xFFFF0001, 300, 4)]:
        hc.uthc_philox(seed, cand, stream, rnd, op, out)
        want = ph.draw(seed, np.array([cand], dtype=np.uint64), stream, rnd, op)
        assert list(out) == [int(w[0]) for w in want]


def _batch(lib, name, xs):
    fn = getattr(lib, name)
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_longlong]
    x = np.ascontiguousarray(xs, dtype=np.float64)
    out = np.empty_like(x)
    fn(x.ctypes.data, out.ctypes.data, x.size)
    return out


def test_py_log2_matches_cpython(hc):
    """ut::libm_log / py_log2 restate glibc's __log_fma (the log CPython's
    math.log calls here) bit for bit: LogIntegerParameter._scale =
    math.log(v + 1.0 - min, 2.0) (manipulator.py:784-787) on every integer
    argument in [1, 2^22], 10^6 random integers below 2^31, integers near 2^53,
    and random positive doubles (subnormals and the |x - 1| < 1/16 branch
    included).  This is what removes the LogInteger table-size limit on
    bit-exact digests."""
    rng = random.Random(7)
    ints = np.arange(1, (1 << 22) + 1, dtype=np.float64)
    rnd = np.array([rng.randrange(1, 1 << 31) for _ in range(1000000)], dtype=np.float64)
    big = np.array([2.0 ** 53 - k for k in range(1, 2000)] + [float(rng.randrange(1 << 31, 1 << 53))
                                                               for _ in range(100000)])
    bits = np.array([rng.getrandbits(63) for _ in range(200000)], dtype=np.uint64).view(np.float64)
    bits = bits[np.isfinite(bits) & (bits > 0)]
    near1 = np.array([1.0 + rng.uniform(-0.0625, 0.0647) for _ in range(100000)])
    special = np.array([0.5001, 1.4999, 2.4999, 1e6 + 0.4999, 5e-324, 2.2250738585072014e-308, 1.7976931348623157e308,
                        1.0, 0.9375, float.fromhex("0x1.09p+0"), float("inf")])
    for xs in (ints, rnd, big, bits, near1, special):
        got = _batch(hc, "uthc_py_log2", xs)
        want = np.array([math.log(x, 2.0) for x in xs.tolist()])
        bad = np.flatnonzero(got.view(np.uint64) != want.view(np.uint64))
        assert bad.size == 0, [(xs[i], got[i], want[i]) for i in bad[:5]]
        gl = _batch(hc, "uthc_libm_log", xs)
        wl = np.array([math.log(x) for x in xs.tolist()])
        assert np.array_equal(gl.view(np.uint64), wl.view(np.uint64))
    # domain edges of log itself
    assert _batch(hc, "uthc_libm_log", [0.0])[0] == float("-inf")
    assert math.isnan(_batch(hc, "uthc_libm_log", [-1.0])[0])


def test_libm_log_fixture_cases(hc):
    """tests/golden/libm_log_non_cr.json: arguments where glibc's log is not
    correctly rounded (confirmed here with Decimal); the restatement follows
    glibc there too"""
    import json
    from decimal import Decimal, getcontext
    getcontext().prec = 60
    xs = json.load(open(os.path.join(ROOT, "tests", "golden", "libm_log_non_cr.json")))["ints"]
    assert len(xs) >= 200
    for x in xs[:40]:
        assert math.log(x) != float(Decimal(x).ln())
    got = _batch(hc, "uthc_py_log2", [float(x) for x in xs])
    assert got.tolist() == [math.log(float(x), 2.0) for x in xs]


def test_logint_unscale_matches_cpython(hc):
    """LogIntegerParameter._unscale int(round(2.0 ** v - 1.0 + min))
    (manipulator.py:787-790): the device's correctly rounded 2^v gives the same
    stored integer as CPython's pow on every argument tried"""
    rng = random.Random(8)
    for mn, mx in ((1.0, 1024.0), (0.0, 1e6), (5.0, 3e9), (1.0, 2.0 ** 40)):
        lo = math.log(mn - 0.4999 + 1.0 - mn, 2.0)
        hi = math.log(mx + 0.4999 + 1.0 - mn, 2.0)
        xs = np.array([rng.uniform(lo, hi) for _ in range(100000)] + [lo, hi])
        got = _batch_unscale(hc, xs, mn)
        want = np.array([float(int(round(2.0 ** float(x) - 1.0 + mn))) for x in xs])
        assert np.array_equal(got, want)


def _batch_unscale(lib, xs, mn):
    fn = lib.uthc_logint_unscale
    fn.argtypes = [ctypes.c_void_p, ctypes.c_double, ctypes.c_void_p, ctypes.c_longlong]
    x = np.ascontiguousarray(xs, dtype=np.float64)
    out = np.empty_like(x)
    fn(x.ctypes.data, mn, out.ctypes.data, x.size)
    return out
