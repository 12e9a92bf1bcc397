"""Dedup and top-k selection semantics.

dedup: a candidate is a duplicate when its hash_config
digest is in the results history (driver.py:157-158, 253-258;
resultsdb/models.py:126-135; api.py:254-280) or an earlier candidate (smaller
global index) of the same batch has the same digest.

top-k (a8): sorted(valid, key=lambda i: (-score[i], i))[:k]; NaN and
duplicate candidates are never selected; missing slots are -1.
"""
import math


def dedup(digests, history):
    hist = set(history)
    seen = set()
    out = []
    for d in digests:
        if d in hist or d in seen:
            out.append(1)
        else:
            out.append(0)
        seen.add(d)
    return out


def topk(scores, k, dup=None, cand_base=0):
    valid = [i for i, s in enumerate(scores)
             if not (dup is not None and dup[i]) and not (isinstance(s, float) and math.isnan(s))]
    valid.sort(key=lambda i: (-scores[i], i))
    sel = [cand_base + i for i in valid[:k]]
    return sel + [-1] * (k - len(sel))
