"""Host-side logic (CPU): C ABI exports, space compilation, value codecs."""
import ctypes
import hashlib
import os
import re

import numpy as np
import pytest

from uptune_amd import _lib as L
from uptune_amd.manipulator import (BooleanParameter, ConfigurationManipulator, EnumParameter, FloatParameter,
                                    IntegerParameter, compile_space, to_descs, unit_bounds)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    src = open(os.path.join(ROOT, "include", "uthot.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(ut_\w+)\s*\(", src, flags=re.M)))


def test_library_exports_every_header_symbol():
    lib = L.lib()
    syms = header_symbols()
    assert len(syms) >= 25
    for s in syms:
        assert hasattr(lib, s), s
        assert s in L.SIGNATURES, s
    assert lib.ut_version() == 1


def test_ctx_create_fails_loudly_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    p = ctypes.c_void_p()
    assert L.lib().ut_ctx_create(0, 0, ctypes.byref(p)) == -2
    from uptune_amd.engine import BatchEngine
    with pytest.raises(L.UthotError):
        BatchEngine([FloatParameter("x", 0.0, 1.0)])


def test_struct_layouts():
    """ctypes mirrors == the C compiler's layout of include/uthot.h (host build)"""
    import os
    hc = ctypes.CDLL(os.path.join(os.path.dirname(L.LIB_PATH), "libuthot_hostcheck.so"))
    hc.uthc_sizeof.restype = ctypes.c_longlong
    for i, st in enumerate([L.ParamDesc, L.GpHyper, L.RoundOut, L.DeParams, L.Acq, L.PsoParams, L.GaParams,
                            L.TreeNode, L.PruneStats]):
        assert ctypes.sizeof(st) == hc.uthc_sizeof(i), st.__name__
    assert ctypes.sizeof(L.ParamDesc) == 112


def test_compile_space_mixed():
    m = ConfigurationManipulator()
    m.add_parameter(FloatParameter("b", -5, 5))
    m.add_parameter(IntegerParameter("a", 1, 10))
    m.add_parameter(BooleanParameter("c"))
    m.add_parameter(EnumParameter("d", ["on", "off", 3]))
    spec = compile_space(m)
    assert spec.order == [1, 0, 2, 3]
    assert spec.n_features == 1 + 1 + 1 + 3
    assert [p.feat_col for p in spec.params] == [0, 1, 2, 3]
    a = spec.params[1]
    assert (a.u_lo, a.u_hi) == (1 - 0.4999, 10 + 0.4999)
    assert a.u_span == float((10 + 0.4999) - (1 - 0.4999))
    assert len(a.lut) == 10 * 32 and a.lut[:32] == hashlib.sha256(b"1").digest()
    d = spec.params[3]
    assert d.lut[64:96] == hashlib.sha256(repr(3).encode()).digest()
    assert spec.params[2].lut[:32] == hashlib.sha256(b"False").digest()
    cfgs = [{"b": 1.5, "a": 3, "c": True, "d": 3}, {"b": -5.0, "a": 10, "c": False, "d": "on"}]
    vals = spec.encode_configs(cfgs)
    np.testing.assert_array_equal(vals[:, 0], [1.5, 3.0, 1.0, 2.0])
    assert spec.decode_values(vals) == cfgs
    descs, keep = to_descs(spec)
    assert descs[1].sort_rank == 0 and descs[0].sort_rank == 1
    assert descs[3].lut_count == 3 and descs[0].lut_count == 0


def test_unit_bounds_python_arithmetic():
    lo, hi, span = unit_bounds(L.UT_INT, 0, 3)
    assert lo == 0 - 0.4999 and hi == 3 + 0.4999 and span == float(hi - lo)
    lo, hi, span = unit_bounds(L.UT_FLOAT, -1000.0, 1000.0)
    assert span == 2000.0


def test_duck_typed_reference_like_params():
    class IntegerParameter:  # noqa: N801 - mimics the reference class name
        def __init__(self, name, lo, hi):
            self.name, self.min_value, self.max_value = name, lo, hi

    spec = compile_space([IntegerParameter("BLOCK_SIZE", 1, 10)])
    assert spec.params[0].kind == L.UT_INT and spec.params[0].lo == 1.0


def test_compile_space_scaled_kinds():
    """LogInteger / PowerOfTwo descriptors carry the reference's legal ranges
    (manipulator.py:792-795, :829-830) and host-computed CPython tables"""
    import math
    from uptune_amd import spaces
    from uptune_amd import _lib as L
    from uptune_amd.manipulator import LOGINT_TABLE_MAX, compile_space, to_descs
    spec = compile_space(spaces.hpl64())
    assert spec.P == 64
    by = {ps.name: ps for ps in spec.params}
    li = by["logint_2"]
    assert li.kind == L.UT_LOGINT and (li.lo, li.hi) == (16.0, 65536.0)
    assert li.u_lo == math.log(16.0 - 0.4999 + 1.0 - 16.0, 2.0)
    assert li.u_hi == math.log(65536.0 + 0.4999 + 1.0 - 16.0, 2.0)
    assert li.vtab.size == 65536 - 16 + 1 and li.vtab[5] == math.log(21 + 1.0 - 16.0, 2.0)
    assert len(li.lut) == 32 * li.vtab.size
    assert by["logint_3"].vtab is None and (1 << 30) + 1 > LOGINT_TABLE_MAX    # device log
    p2 = by["pow2_1"]
    assert p2.kind == L.UT_POW2 and (p2.u_lo, p2.u_hi) == (4 - 0.4999, 20 + 0.4999) and len(p2.lut) == 32 * 17
    arr, keep = to_descs(spec)
    assert arr[[i for i, ps in enumerate(spec.params) if ps.name == "logint_2"][0]].vtab_count == 65521
    cfg = {"pow2_1": 1 << 9, "logint_2": 300}
    assert by["pow2_1"].to_value(cfg["pow2_1"]) == 512.0 and by["logint_2"].from_value(300.0) == 300


def test_encode_decode_ints_beyond_int64():
    """INT values of magnitude >= 2^63 take the per-value float(int(v)) /
    int(x) path: no OverflowError on encode, no int64 wrap on decode"""
    m = ConfigurationManipulator([IntegerParameter("big", -(1 << 70), 1 << 70), FloatParameter("x", 0.0, 1.0)])
    spec = compile_space(m)
    cfgs = [{"big": 1 << 65, "x": 0.5}, {"big": -(1 << 64) - 12345, "x": 0.25}, {"big": 7, "x": 1.0}]
    vals = spec.encode_configs(cfgs)
    assert vals[0].tolist() == [float(1 << 65), float(-(1 << 64) - 12345), 7.0]
    back = spec.decode_values(vals)
    assert [c["big"] for c in back] == [int(float(1 << 65)), int(float(-(1 << 64) - 12345)), 7]
    assert [c["x"] for c in back] == [0.5, 0.25, 1.0]
