"""Parameter kinds and their value arithmetic, restated from
python/uptune/opentuner/search/manipulator.py.

A space is a list of `Param`; a configuration row is a list of stored
values (FLOAT float, INT int, LOGINT int, POW2 int power of two, BOOL bool,
ENUM the option object).  Scalar functions follow the reference line by line
(Python floats, Python round/min/max, math.log, float **); the *_vec versions
are the same arithmetic over numpy float64 columns (elementwise IEEE ops,
np.rint == Python round half-even; the two libm calls of the scaled kinds,
math.log and 2.0 ** v, stay CPython's own, element by element), checked equal
to the scalar versions in tests/test_oracle.py.

Scaled kinds (ScaledNumericParameter, manipulator.py:747-775): the value
searched on (get_value) is a transform of the stored value:
  LOGINT  LogIntegerParameter  manipulator.py:778-797 (a FloatParameter: value_type float)
          get_value = math.log(v + 1.0 - min, 2.0)          (_scale   :784-785)
          set_value(s) stores int(round(2.0 ** s - 1.0 + min))  (_unscale :787-790)
          legal_range = (_scale(min - 0.4999), _scale(max + 0.4999))  (:792-795)
  POW2    PowerOfTwoParameter  manipulator.py:811-836 (an IntegerParameter)
          get_value = int(math.log(v, 2)) (the exponent)    (:823-824)
          set_value(e) stores 2 ** int(e)                    (:826-827)
          legal_range = (int(log2 min), int(log2 max))       (:829-830)
"""
import math
from dataclasses import dataclass, field
from typing import Any, List

import numpy as np

FLOAT, INT, LOGINT, POW2, BOOL, ENUM, PERM = range(7)


@dataclass
class Param:
    name: Any
    kind: int
    lo: Any = 0          # min_value as given (LOGINT/POW2: the stored bounds)
    hi: Any = 0
    options: List[Any] = field(default_factory=list)

    def is_primitive(self):
        return self.kind in (FLOAT, INT, LOGINT, POW2)

    def is_integer_type(self):
        # value_type(0) == value_type(0.1)  manipulator.py:469-471
        return self.kind in (INT, POW2)

    def legal_range(self):
        if self.kind == LOGINT:
            lo, hi = float(self.lo), float(self.hi)          # FloatParameter stores floats
            return scale(self, lo - 0.4999), scale(self, hi + 0.4999)
        if self.kind == POW2:
            return int(math.log(self.lo, 2)), int(math.log(self.hi, 2))
        # NumericParameter.legal_range  manipulator.py:593-594
        return self.lo, self.hi


def scale(p, v):
    """get_value of a stored value (ScaledNumericParameter._scale)"""
    if p.kind == LOGINT:
        return math.log(v + 1.0 - float(p.lo), 2.0)
    if p.kind == POW2:
        return int(math.log(v, 2))
    return v


def unscale(p, s):
    """stored value of a searched value (ScaledNumericParameter._unscale)"""
    if p.kind == LOGINT:
        return int(round(2.0 ** s - 1.0 + float(p.lo)))
    if p.kind == POW2:
        return 2 ** int(s)
    return s


def unit_range(p):
    """low/high used by get/set_unit_value (manipulator.py:475-479)"""
    low, high = p.legal_range()
    if p.is_integer_type():
        low -= 0.4999
        high += 0.4999
    return low, high


def get_unit_value(p, raw):
    """manipulator.py:473-488 (raw = the stored value)"""
    low, high = unit_range(p)
    val = scale(p, raw)
    if low < high:
        return float(val - low) / float(high - low)
    return 0.0


def set_unit_value(p, unit_value, current):
    """manipulator.py:490-503 -> new stored value (current if unchanged)"""
    assert 0.0 <= unit_value <= 1.0
    low, high = unit_range(p)
    if low < high:
        val = unit_value * float(high - low) + low
        if p.is_integer_type():
            val = round(val)
        val = max(low, min(val, high))
        val = int(val) if p.is_integer_type() else float(val)   # self.value_type(val)
        return unscale(p, val)                                 # set_value -> _unscale
    return current


def op4_set_linear_primitive(p, va_raw, vb_raw, vc_raw, a, b, c, current):
    """PrimitiveParameter.op4_set_linear  manipulator.py:523-542"""
    va = get_unit_value(p, va_raw)
    vb = get_unit_value(p, vb_raw)
    vc = get_unit_value(p, vc_raw)
    v = a * va + b * vb + c * vc
    v = max(0.0, min(v, 1.0))
    return set_unit_value(p, v, current)


def randomize(p, x, y, z, w):
    """op1_randomize given one Philox block (x, y, z, w) as Python ints.
    FLOAT:  random.uniform(lo, hi) = lo + (hi-lo)*random()   manipulator.py:606
    INT:    random.randint(lo, hi)                            manipulator.py:604
    LOGINT: set_value(uniform(*legal_range))  (not integer-typed)  :603-606
    POW2:   set_value(randint(*legal_range))  (integer-typed)      :603-604
    BOOL:   random.choice((True, False))                      manipulator.py:946-949
    ENUM:   random.choice(options)                            manipulator.py:1039
    """
    from . import philox as ph
    if p.kind in (FLOAT, LOGINT):
        lo, hi = p.legal_range()
        u = float(ph.u01(x, y))
        return unscale(p, lo + (hi - lo) * u)
    r64 = int(ph.u64(z, w))
    if p.kind in (INT, POW2):
        lo, hi = p.legal_range()
        return unscale(p, lo + (r64 * (hi - lo + 1) >> 64))
    if p.kind == BOOL:
        return (True, False)[(r64 * 2) >> 64]
    if p.kind == ENUM:
        return p.options[(r64 * len(p.options)) >> 64]
    raise NotImplementedError(p.kind)


# ---- SoA column layout: a PERM of size S owns S columns of item indices ----
def width(p):
    return len(p.options) if p.kind == PERM else 1


def columns(space):
    """first SoA column of every param, and the column count"""
    cols, c = [], 0
    for p in space:
        cols.append(c)
        c += width(p)
    return cols, c


def row_values(space, soa, j):
    """stored values of candidate j (PERM: the list of items)"""
    cols, _ = columns(space)
    out = []
    for p, c in zip(space, cols):
        if p.kind == PERM:
            out.append([p.options[int(x)] for x in soa[c:c + width(p), j]])
        else:
            out.append(from_f64(p, soa[c, j]))
    return out


def soa_from_rows(space, rows):
    """list of stored-value rows -> SoA [ncols][n]"""
    cols, nc = columns(space)
    out = np.empty((nc, len(rows)))
    for j, row in enumerate(rows):
        for p, c, v in zip(space, cols, row):
            if p.kind == PERM:
                idx = {repr(it): k for k, it in enumerate(p.options)}
                out[c:c + width(p), j] = [idx[repr(it)] for it in v]
            else:
                out[c, j] = to_f64(p, v)
    return out


# ---- value <-> f64 column codec (the device's SoA representation) --------
def to_f64(p, v):
    if p.kind == FLOAT:
        return float(v)
    if p.kind in (INT, LOGINT, POW2):
        return float(int(v))
    if p.kind == BOOL:
        return 1.0 if v else 0.0
    if p.kind == ENUM:
        return float(p.options.index(v))
    raise NotImplementedError(p.kind)


def from_f64(p, x):
    if p.kind == FLOAT:
        return float(x)
    if p.kind in (INT, LOGINT, POW2):
        return int(x)
    if p.kind == BOOL:
        return bool(x != 0.0)
    if p.kind == ENUM:
        return p.options[int(x)]
    raise NotImplementedError(p.kind)


# ---- vectorised forms over f64 columns -----------------------------------
def unit_consts(p):
    low, high = unit_range(p)
    return float(low), float(high), float(high - low)


def scale_vec(p, col):
    if p.kind == LOGINT:
        lo = float(p.lo)
        return np.array([math.log(float(v) + 1.0 - lo, 2.0) for v in np.ravel(col)]).reshape(np.shape(col))
    if p.kind == POW2:
        return np.frexp(col)[1].astype(np.float64) - 1.0    # exact log2 of a power of two
    return col


def unscale_vec(p, s):
    if p.kind == LOGINT:
        return np.array([float(unscale(p, float(v))) for v in np.ravel(s)]).reshape(np.shape(s))
    if p.kind == POW2:
        return np.ldexp(1.0, s.astype(np.int64))
    return s


def get_unit_value_vec(p, col):
    low, high, span = unit_consts(p)
    if low < high:
        return (scale_vec(p, col) - low) / span
    return np.zeros_like(col)


def set_unit_value_vec(p, u, current):
    low, high, span = unit_consts(p)
    if not (low < high):
        return current.copy()
    val = u * span + low
    if p.is_integer_type():
        val = np.rint(val)
    val = np.where(high < val, high, val)   # min(val, high)
    val = np.where(val > low, val, low)     # max(low, .)
    if p.is_integer_type():
        val = np.trunc(val)
    return unscale_vec(p, val)


def features(space, rows_f64):
    """GP features of SoA rows [ncols][n]: unit values, BOOL 0/1, ENUM one-hot,
    PERM position of each item / (S - 1) (the build's encoding, SURVEY.md
    §8(a) GP spec: "Perm ... position-normalised")."""
    cols = []
    starts, _ = columns(space)
    for p, c0 in zip(space, starts):
        col = rows_f64[c0]
        if p.kind == PERM:
            S = width(p)
            pos = np.zeros((S, rows_f64.shape[1]))
            for k in range(S):
                items = rows_f64[c0 + k].astype(np.int64)
                pos[items, np.arange(rows_f64.shape[1])] = (k / (S - 1)) if S > 1 else 0.0
            cols.extend(list(pos))
            continue
        if p.is_primitive():
            cols.append(get_unit_value_vec(p, col))
        elif p.kind == BOOL:
            cols.append(col.copy())
        elif p.kind == ENUM:
            for k in range(len(p.options)):
                cols.append((col == k).astype(np.float64))
    return np.stack(cols)
