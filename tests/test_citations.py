"""Every `name.py:N[-M]` citation of the reference in the product, the oracle,
the C-ABI header and the integration notes points inside the cited file
(citations past the end of pso.py / globalGA.py).

The reference tree is read as text (line counts only); the test is skipped
where it is absent (the GPU box).  A citation resolves to the reference files
of that basename, narrowed by its path when it has one (`OT/` =
python/uptune/opentuner/, `PY/` = python/uptune/); names no reference file
carries (this repository's own files, CPython's stdlib) are not checked.
"""
import os
import re

import pytest

REF = "/root/reference"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CITE = re.compile(r"((?:[\w.]+/)*\w+\.py):(\d+)(?:-(\d+))?")
SCOPE = ("oracle", "include", "uptune_amd")
DOCS = ("INTEGRATION.md", "DESIGN.md")


def _ref_files():
    out = {}
    for dp, dn, fn in os.walk(REF):
        dn[:] = [d for d in dn if d != ".git"]
        for f in fn:
            if f.endswith(".py"):
                p = os.path.join(dp, f)
                with open(p, errors="replace") as fh:
                    n = sum(1 for _ in fh)
                out.setdefault(f, []).append((os.path.relpath(p, REF), n))
    return out


def _sources():
    for d in SCOPE:
        for dp, dn, fn in os.walk(os.path.join(ROOT, d)):
            dn[:] = [x for x in dn if x not in ("_build", "__pycache__", "_ref")]
            for f in fn:
                if f.endswith((".py", ".h", ".hip", ".cpp")):
                    yield os.path.join(dp, f)
    for f in DOCS:
        yield os.path.join(ROOT, f)


@pytest.mark.skipif(not os.path.isdir(REF), reason="the reference tree is not present here")
def test_reference_citations_in_range():
    ref = _ref_files()
    checked, bad = 0, []
    for path in _sources():
        with open(path, errors="replace") as fh:
            for ln, line in enumerate(fh, 1):
                for mm in CITE.finditer(line):
                    cited, a = mm.group(1), int(mm.group(2))
                    b = int(mm.group(3) or a)
                    cands = ref.get(os.path.basename(cited))
                    if not cands:
                        continue
                    full = cited.replace("OT/", "python/uptune/opentuner/").replace("PY/", "python/uptune/")
                    sel = [c for c in cands if c[0].endswith(full)] or cands
                    longest = max(n for _, n in sel)
                    checked += 1
                    if a < 1 or b < a or b > longest:
                        bad.append(f"{os.path.relpath(path, ROOT)}:{ln}: {mm.group(0)} "
                                   f"(longest match {longest} lines: {[c[0] for c in sel]})")
    assert checked > 100, checked
    assert not bad, "\n".join(bad)
