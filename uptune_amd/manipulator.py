"""Host-side mirror of the reference's search-space API.

Same class names, constructor arguments and value semantics as
python/uptune/opentuner/search/manipulator.py (the parameter kinds that
uptune's create_params builds, python/uptune/api.py:179-199):

    IntegerParameter(name, min, max)          manipulator.py:651
    FloatParameter(name, min, max)            manipulator.py:703
    LogIntegerParameter(name, min, max)       manipulator.py:781
    PowerOfTwoParameter(name, min, max)       manipulator.py:813
    BooleanParameter(name)                    manipulator.py:930
    EnumParameter(name, options)              manipulator.py:1024
    PermutationParameter(name, items)         manipulator.py:1048
    ConfigurationManipulator(params)          manipulator.py:129

A configuration is a plain dict name -> value, exactly as in the reference.
The batch work (proposal, hash_config, dedup, scoring) runs on the GPU via
uptune_amd.engine.BatchEngine; this module only describes the space and
converts between config dicts and the device's structure-of-arrays rows.

`compile_space` also accepts a reference ConfigurationManipulator (duck
typed on class names and min_value/max_value/options attributes), which is
what makes the GPU techniques a drop-in for an existing OpenTuner/uptune
search driver.
"""
from __future__ import annotations

import hashlib
import math
import operator
from dataclasses import dataclass, field
from typing import Any, Dict, List, Sequence

import numpy as np

from . import _lib as L

# discrete INT ranges up to this many values get an inner-digest LUT
INT_LUT_MAX = 4096
# LogInteger ranges up to this many values get host tables (get_value and the
# precomputed inner digest sha256(repr(get_value)), which saves the device one
# repr + SHA-256 per value).  Larger ranges compute get_value on the device
# with ut_core.h libm_log, a bit-exact restatement of the glibc log CPython's
# math.log calls (tests/test_core_host.py test_py_log2_matches_cpython), so
# both paths give the reference's values and digests.
LOGINT_TABLE_MAX = 1 << 22


class Parameter:
    """Base of the mirrored parameter kinds (manipulator.py:275)."""

    def __init__(self, name):
        self.name = name
        self.parent = None

    def is_primitive(self, ignored=None) -> bool:
        return isinstance(self, PrimitiveParameter)

    def is_permutation(self, ignored=None) -> bool:
        return isinstance(self, PermutationParameter)


class PrimitiveParameter(Parameter):
    value_type: type = float

    def is_integer_type(self) -> bool:
        return self.value_type(0) == self.value_type(0.1)


class NumericParameter(PrimitiveParameter):
    def __init__(self, name, min_value, max_value):
        assert min_value <= max_value
        super().__init__(name)
        self.min_value = self.value_type(min_value)
        self.max_value = self.value_type(max_value)

    def legal_range(self, config=None):
        return self.min_value, self.max_value


class IntegerParameter(NumericParameter):
    value_type = int


class FloatParameter(NumericParameter):
    value_type = float


class LogIntegerParameter(FloatParameter):
    """integer searched on a log scale (manipulator.py:778-797): stored as an
    int, get_value = math.log(v + 1.0 - min, 2.0)."""

    def __init__(self, name, min_value, max_value):
        Parameter.__init__(self, name)
        self.min_value = float(min_value)
        self.max_value = float(max_value)

    def _scale(self, v):
        return math.log(v + 1.0 - self.min_value, 2.0)

    def _unscale(self, v):
        return int(round(2.0 ** v - 1.0 + self.min_value))

    def legal_range(self, config=None):
        return self._scale(self.min_value - 0.4999), self._scale(self.max_value + 0.4999)


class PowerOfTwoParameter(IntegerParameter):
    """power of two searched by exponent (manipulator.py:811-836)."""

    def legal_range(self, config=None):
        return int(math.log(self.min_value, 2)), int(math.log(self.max_value, 2))

    def __init__(self, name, min_value, max_value):
        assert min_value >= 1
        assert math.log(min_value, 2) % 1 == 0
        assert math.log(max_value, 2) % 1 == 0
        super().__init__(name, min_value, max_value)


class ComplexParameter(Parameter):
    pass


class BooleanParameter(ComplexParameter):
    pass


class EnumParameter(ComplexParameter):
    def __init__(self, name, options):
        super().__init__(name)
        self.options = list(options)


class PermutationParameter(ComplexParameter):
    """ordering of `items` (manipulator.py:1048-1356); on the device a value is
    `size` SoA columns of item indices."""

    def __init__(self, name, items):
        super().__init__(name)
        self._items = list(items)
        self.size = len(items)


class ConfigurationManipulator:
    """Fixed list of parameters; configs are dicts (manipulator.py:129-272)."""

    def __init__(self, params=None, config_type=dict, seed_config=None):
        self.params = list(params or [])
        self.config_type = config_type
        self._seed_config = seed_config
        for p in self.params:
            p.parent = self

    def add_parameter(self, p):
        p.parent = self
        self.params.append(p)

    def parameters(self, config=None):
        return self.params

    def param_names(self, *args):
        return sorted(p.name for p in self.params)

    def copy(self, config):
        import copy
        return copy.deepcopy(config)

    def hash_config(self, config) -> str:
        """sha256 hex identity of a config (manipulator.py:233-243), computed on
        the GPU (batch of one)."""
        from .engine import default_engine
        return default_engine(self).hash_configs([config])[0]


# ---------------------------------------------------------------------------
# space compilation: parameters -> ut_param_desc[] + value codecs
# ---------------------------------------------------------------------------
def _kind_of(p) -> int:
    cls = type(p).__name__
    names = {c.__name__ for c in type(p).__mro__}
    if "PermutationParameter" in names:
        return L.UT_PERM
    if "PowerOfTwoParameter" in names:
        return L.UT_POW2
    if "LogIntegerParameter" in names:
        return L.UT_LOGINT
    if "BooleanParameter" in names:
        return L.UT_BOOL
    if "EnumParameter" in names:
        return L.UT_ENUM
    if "IntegerParameter" in names:
        return L.UT_INT
    if "FloatParameter" in names:
        return L.UT_FLOAT
    raise TypeError(f"unsupported parameter class {cls} for {getattr(p, 'name', '?')!r}")


def _digest(s: str) -> bytes:
    return hashlib.sha256(s.encode("utf-8")).digest()


@dataclass
class ParamSpec:
    name: Any
    kind: int
    lo: float = 0.0
    hi: float = 0.0
    u_lo: float = 0.0
    u_hi: float = 0.0
    u_span: float = 0.0
    options: List[Any] = field(default_factory=list)
    feat_col: int = 0
    n_feat: int = 1
    col: int = 0          # first SoA value column
    width: int = 1        # SoA columns (PERM: its size)
    lut: bytes = b""
    vtab: Any = None      # LOGINT: float64 get_value table

    def to_columns(self, v) -> List[float]:
        """stored value -> its SoA column values"""
        if self.kind == L.UT_PERM:
            index = {repr(it): k for k, it in enumerate(self.options)}
            return [float(index[repr(it)]) for it in v]
        return [self.to_value(v)]

    def from_columns(self, xs):
        if self.kind == L.UT_PERM:
            return [self.options[int(x)] for x in xs]
        return self.from_value(xs[0])

    def to_value(self, v) -> float:
        if self.kind == L.UT_FLOAT:
            return float(v)
        if self.kind in (L.UT_INT, L.UT_LOGINT, L.UT_POW2):
            return float(int(v))
        if self.kind == L.UT_BOOL:
            return 1.0 if v else 0.0
        if self.kind == L.UT_ENUM:
            return float(self.options.index(v))
        raise TypeError("unsupported kind")

    def from_value(self, x: float):
        if self.kind == L.UT_FLOAT:
            return float(x)
        if self.kind in (L.UT_INT, L.UT_LOGINT, L.UT_POW2):
            return int(x)
        if self.kind == L.UT_BOOL:
            return bool(x != 0.0)
        if self.kind == L.UT_ENUM:
            return self.options[int(x)]
        raise TypeError("unsupported kind")


@dataclass
class SpaceSpec:
    params: List[ParamSpec]
    order: List[int]           # sorted position -> param index
    n_features: int

    @property
    def P(self) -> int:
        return len(self.params)

    @property
    def ncols(self) -> int:
        return sum(p.width for p in self.params)

    def names(self) -> List[Any]:
        return [p.name for p in self.params]

    def encode_configs(self, cfgs: Sequence[Dict[Any, Any]]) -> np.ndarray:
        """configs -> SoA [ncols][n] float64 (ParamSpec.to_columns, column by
        column: one C-level conversion per parameter instead of one Python call
        per value -- a 4096 x 64 seed design in ~10 ms instead of ~0.2 s)"""
        n = len(cfgs)
        out = np.empty((self.ncols, n), dtype=np.float64)   # canonical strides (ld = n)
        if n == 0:
            return out
        # rows of values in parameter order, transposed to columns (C-level loops)
        get = operator.itemgetter(*self.names())
        cols = list(zip(*map(get, cfgs))) if self.P > 1 else [tuple(map(get, cfgs))]
        for ps, col in zip(self.params, cols):
            c0 = ps.col
            if ps.kind == L.UT_FLOAT:
                out[c0] = np.fromiter(map(float, col), dtype=np.float64, count=n)
            elif ps.kind in (L.UT_INT, L.UT_LOGINT, L.UT_POW2):
                try:
                    out[c0] = np.fromiter(map(int, col), dtype=np.int64, count=n)
                except OverflowError:   # |v| >= 2^63: float(int(v)) per value, as to_value does
                    out[c0] = np.fromiter(map(ps.to_value, col), dtype=np.float64, count=n)
            elif ps.kind == L.UT_BOOL:
                out[c0] = np.fromiter(map(bool, col), dtype=bool, count=n)
            elif ps.kind == L.UT_ENUM:
                out[c0] = _enum_indices(ps.options, col)
            else:   # PERM: a value per item
                for j, v in enumerate(col):
                    out[c0:c0 + ps.width, j] = ps.to_columns(v)
        return out

    def decode_values(self, values: np.ndarray) -> List[Dict[Any, Any]]:
        """SoA [ncols][n] -> configs (ParamSpec.from_columns, column by column)"""
        v = np.asarray(values, dtype=np.float64)
        cols = []
        for ps in self.params:
            x = v[ps.col]
            if ps.kind == L.UT_FLOAT:
                cols.append(x.tolist())
            elif ps.kind in (L.UT_INT, L.UT_LOGINT, L.UT_POW2):
                if x.size and not (np.all(np.abs(x) < 2.0 ** 63)):   # int64 would wrap: int(x) per value
                    cols.append([ps.from_value(a) for a in x.tolist()])
                else:
                    cols.append(x.astype(np.int64).tolist())
            elif ps.kind == L.UT_BOOL:
                cols.append((x != 0.0).tolist())
            elif ps.kind == L.UT_ENUM:
                opts = ps.options
                cols.append([opts[i] for i in x.astype(np.int64).tolist()])
            else:
                cols.append([ps.from_columns(r) for r in v[ps.col:ps.col + ps.width].T.tolist()])
        names = self.names()
        return [dict(zip(names, vals)) for vals in zip(*cols)]


def _enum_indices(options, col) -> np.ndarray:
    """[options.index(v) for v in col]: one C-level dict lookup per value when
    every option and value is hashable (first occurrence, the same equality),
    else the list method (which raises ValueError for an unknown value)"""
    try:
        d = {}
        for i, o in enumerate(options):
            d.setdefault(o, i)
        return np.fromiter(map(d.__getitem__, col), dtype=np.int64, count=len(col))
    except (KeyError, TypeError):
        return np.fromiter(map(options.index, col), dtype=np.int64, count=len(col))


def unit_bounds(kind: int, lo, hi):
    """legal range for get/set_unit_value exactly as Python computes it
    (manipulator.py:475-479, 493-497)."""
    low, high = lo, hi
    if kind == L.UT_INT:
        low -= 0.4999
        high += 0.4999
    return float(low), float(high), float(high - low)


def compile_space(params) -> SpaceSpec:
    """Build the device description of a parameter list (our mirror classes or
    the reference's own Parameter objects)."""
    if hasattr(params, "params"):
        params = params.params
    specs: List[ParamSpec] = []
    feat = 0
    col = 0
    for p in params:
        kind = _kind_of(p)
        ps = ParamSpec(name=p.name, kind=kind)
        if kind in (L.UT_FLOAT, L.UT_INT):
            lo, hi = p.min_value, p.max_value
            ps.lo, ps.hi = float(lo), float(hi)
            ps.u_lo, ps.u_hi, ps.u_span = unit_bounds(kind, lo, hi)
            ps.n_feat = 1
            if kind == L.UT_INT and (hi - lo + 1) <= INT_LUT_MAX:
                ps.lut = b"".join(_digest(repr(int(v))) for v in range(int(lo), int(hi) + 1))
        elif kind == L.UT_LOGINT:
            # LogIntegerParameter (manipulator.py:778-797): stored int bounds,
            # searched on log2 values over the widened legal_range
            mn, mx = float(p.min_value), float(p.max_value)
            ps.lo, ps.hi = mn, mx
            scale = lambda v: math.log(v + 1.0 - mn, 2.0)  # noqa: E731  (_scale :784-785)
            ps.u_lo, ps.u_hi = scale(mn - 0.4999), scale(mx + 0.4999)
            ps.u_span = float(ps.u_hi - ps.u_lo)
            n = int(mx) - int(mn) + 1
            if n <= LOGINT_TABLE_MAX:
                vals = [scale(float(v)) for v in range(int(mn), int(mx) + 1)]
                ps.vtab = np.array(vals, dtype=np.float64)
                ps.lut = b"".join(_digest(repr(x)) for x in vals)
        elif kind == L.UT_POW2:
            # PowerOfTwoParameter (manipulator.py:811-836): searched by the exponent
            ps.lo, ps.hi = float(p.min_value), float(p.max_value)
            elo, ehi = int(math.log(p.min_value, 2)), int(math.log(p.max_value, 2))
            ps.u_lo, ps.u_hi, ps.u_span = unit_bounds(L.UT_INT, elo, ehi)
            ps.lut = b"".join(_digest(repr(e)) for e in range(elo, ehi + 1))
        elif kind == L.UT_BOOL:
            ps.options = [True, False]
            ps.n_feat = 1
            ps.lut = _digest(repr(False)) + _digest(repr(True))
        elif kind == L.UT_ENUM:
            ps.options = list(p.options)
            ps.n_feat = len(ps.options)
            ps.lut = b"".join(_digest(repr(o)) for o in ps.options)
        elif kind == L.UT_PERM:
            # PermutationParameter(name, items): item indices in `size` columns;
            # GP features = each item's position / (size - 1)
            ps.options = list(p._items)
            ps.width = len(ps.options)
            ps.n_feat = len(ps.options)
            if len({repr(it) for it in ps.options}) != len(ps.options):
                raise ValueError(f"permutation {p.name!r}: items must have distinct reprs")
        ps.feat_col = feat
        ps.col = col
        feat += ps.n_feat
        col += ps.width
        specs.append(ps)
    order = sorted(range(len(specs)), key=lambda i: specs[i].name)
    return SpaceSpec(params=specs, order=order, n_features=feat)


def to_descs(spec: SpaceSpec):
    """SpaceSpec -> (ctypes ParamDesc array, keepalive list)"""
    keep = []
    arr = (L.ParamDesc * spec.P)()
    rank = [0] * spec.P
    for r, i in enumerate(spec.order):
        rank[i] = r
    for i, ps in enumerate(spec.params):
        d = arr[i]
        d.kind = ps.kind
        d.sort_rank = rank[i]
        d.lo, d.hi = ps.lo, ps.hi
        d.u_lo, d.u_hi, d.u_span = ps.u_lo, ps.u_hi, ps.u_span
        d.n_options = len(ps.options)
        if ps.kind == L.UT_PERM:
            reprs = [repr(it).encode("utf-8") for it in ps.options]
            rb = np.frombuffer(b"".join(reprs), dtype=np.uint8).copy()
            ro = np.concatenate([[0], np.cumsum([len(r) for r in reprs])]).astype(np.int32)
            keep += [rb, ro]
            d.perm_repr_host = rb.ctypes.data
            d.perm_repr_off_host = ro.ctypes.data
        nb = str(ps.name).encode("utf-8")
        keep.append(nb)
        d.name = nb
        d.name_len = len(nb)
        if ps.lut:
            buf = (np.frombuffer(ps.lut, dtype=np.uint8)).copy()
            keep.append(buf)
            d.lut_count = len(ps.lut) // 32
            d.lut_host = buf.ctypes.data
        else:
            d.lut_count = 0
            d.lut_host = None
        if ps.vtab is not None:
            vt = np.ascontiguousarray(ps.vtab, dtype=np.float64)
            keep.append(vt)
            d.vtab_count = vt.size
            d.vtab_host = vt.ctypes.data
        else:
            d.vtab_count = 0
            d.vtab_host = None
    return arr, keep
