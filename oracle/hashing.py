"""ConfigurationManipulator.hash_config restated
(python/uptune/opentuner/search/manipulator.py:233-243, :456-459, :855-858).

    m = hashlib.sha256()
    params.sort(key=_.name)
    for i, p in enumerate(params):
        m.update(str(p.name).encode())
        m.update(str(p.hash_value(config)).encode())
        m.update(str(i).encode())
        m.update(b"|")

Primitive hash_value returns sha256(repr(get_value(cfg)).encode('utf-8'))
.hexdigest().encode() -- a *bytes* object, so uptune's Python-3 port feeds
str(bytes) = "b'<hex>'" to the outer hash.  Complex params return the str
hexdigest.  py2=True reproduces the original OpenTuner (Python 2) layout in
which both are plain hex (pinned by samples/tutorials/tuneup.opentuner.db).
"""
import hashlib

from .space import BOOL, ENUM, FLOAT, PERM, scale


def hash_value(p, v, py2=False):
    if p.is_primitive():
        # repr(self.get_value(config)): LOGINT hashes its log-scale float,
        # POW2 its integer exponent (ScaledNumericParameter.get_value :769-770)
        gv = scale(p, float(v) if p.kind == FLOAT else int(v))
        inner = hashlib.sha256(repr(gv).encode("utf-8")).hexdigest().encode()
        return inner.decode() if py2 else str(inner)
    if p.kind == BOOL:
        return hashlib.sha256(repr(bool(v)).encode()).hexdigest()
    if p.kind in (ENUM, PERM):   # PERM: v is the list of items, repr(list)
        return hashlib.sha256(repr(v).encode()).hexdigest()
    raise NotImplementedError(p.kind)


def outer_message(space, cfg, py2=False):
    """the exact byte string fed to the outer sha256"""
    order = sorted(range(len(space)), key=lambda i: space[i].name)
    out = []
    for i, j in enumerate(order):
        p = space[j]
        out.append(str(p.name).encode())
        out.append(str(hash_value(p, cfg[j], py2)).encode())
        out.append(str(i).encode())
        out.append(b"|")
    return b"".join(out)


def hash_config(space, cfg, py2=False):
    """cfg: list of stored values, one per param of `space`"""
    return hashlib.sha256(outer_message(space, cfg, py2)).hexdigest()
