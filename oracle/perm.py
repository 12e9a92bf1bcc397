"""PermutationParameter operators restated from
python/uptune/opentuner/search/manipulator.py:1048-1356 (TEST INFRASTRUCTURE:
imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline).

A permutation value is a list of item indices (0..S-1 into the parameter's
`items`).  Every operator below is the reference's list code with its
`random.*` calls replaced by words of a counter-RNG draw site:

    site = (seed, candidate g, stream, round, op)
    block b = Philox4x32-10(counter = (g_lo, g_hi, stream, (round << 8) | (op | 0x80)),
                            key     = (seed_lo, seed_hi ^ b))
    word k  = block (k >> 2), component k & 3   (x, y, z, w)

    randint(a, b)          -> a + randbelow(word, b - a + 1)
    randbelow(word, n)     =  (word * n) >> 32
    random() < p           -> word * 2**-32 < p

which is exactly uptune_amd/csrc/ut_perm.h.  The crossovers take their
randint calls from `ints(W)`: a word stream (the counter form above, call k
reads word k) or any object with randint(a, b) -- CPython's random.Random,
so the same code consumes the reference's MT19937 stream call for call
(oracle/replay.py MTDraws).  Operators and their reference lines:

    op1_randomize            random.shuffle (CPython Fisher-Yates, i = S-1 .. 1)  :1057-1064
    op1_small_random_change  swap (i-1, i) with probability p                    :1066-1079
    op3_cross_PX             :1179-1196     op3_cross_PMX   :1198-1262
    op3_cross_CX             :1264-1302     op3_cross_OX1   :1304-1328
    op3_cross_OX3            :1330-1353
    op3_cross                d = int(round(size * strength))                     :1096-1113
    op3_swarm                U > c: cross with cfg1 if U' < c1 else cfg2          :1115-1140

Edge cases the reference raises on (randint over an empty range: PX with
S < 2, OX/PMX with d > S) leave the base permutation unchanged here.
PMX iterates `candidate_indices` (a set of small ints) in ascending order,
which is CPython's iteration order for a set of non-negative ints smaller
than its table size.  For the crossover sizes the reference uses,
round(0.3 S) (op3_cross) and S // 3 (CrossoverMixin), CPython 3.10 iterates
set(range(r)) | set(range(r + d, S)) in ascending order for every r and
every S < 600 (checked); other d can differ.
"""
from . import philox as ph

PERM_OP_FLAG = 0x80
X_NONE, X_OX1, X_OX3, X_PX, X_CX, X_PMX = range(6)
XNAMES = {"op3_cross_OX1": X_OX1, "op3_cross_OX3": X_OX3, "op3_cross_PX": X_PX, "op3_cross_CX": X_CX,
          "op3_cross_PMX": X_PMX}


class Words:
    """lazy word stream of one draw site (scalar candidate)"""

    def __init__(self, seed, g, stream, round_, op):
        self.seed, self.g, self.stream, self.round_, self.op = int(seed), int(g), int(stream), int(round_), int(op)
        self.blk = {}

    def __getitem__(self, k):
        b = k >> 2
        if b not in self.blk:
            key_hi = ((self.seed >> 32) ^ b) & 0xFFFFFFFF
            c = ph.philox4x32_10(self.g & 0xFFFFFFFF, self.g >> 32, self.stream & 0xFFFFFFFF,
                                 ((self.round_ << 8) | ((self.op | PERM_OP_FLAG) & 0xFF)) & 0xFFFFFFFF,
                                 self.seed & 0xFFFFFFFF, key_hi)
            self.blk[b] = [int(v) for v in c]
        return self.blk[b][k & 3]


def randbelow(word, n):
    return (int(word) * int(n)) >> 32


def randint(word, a, b):
    return a + randbelow(word, b - a + 1)


class WordInts:
    """random.randint(a, b) calls answered from consecutive words of a draw
    site (call k -> word k), the counter form of the crossovers' randint"""

    def __init__(self, W):
        self.W, self.k = W, 0

    def randint(self, a, b):
        v = randint(self.W[self.k], a, b)
        self.k += 1
        return v


def ints(W):
    """the crossovers' randint source: an object with randint(a, b) (e.g.
    CPython's random.Random: the reference's MT19937 stream, in call order) is
    used as it is; a word stream is read one word per call"""
    return W if hasattr(W, "randint") else WordInts(W)


def shuffle(x, W):
    """random.shuffle(x) in place: for i in reversed(range(1, len(x))): j = randbelow(i + 1)"""
    for s, i in enumerate(reversed(range(1, len(x)))):
        j = randbelow(W[s], i + 1)
        x[i], x[j] = x[j], x[i]


def small_random_change(x, W, p=0.25):
    """op1_small_random_change (:1066-1079) in place"""
    for i in range(1, len(x)):
        if W[i - 1] * (1.0 / 4294967296.0) < p:
            x[i - 1], x[i] = x[i], x[i - 1]


def cross_PX(p1, p2, d, W):
    S = len(p1)
    if S < 2:
        return list(p1)
    c1 = ints(W).randint(2, S)
    return sorted(p1[:c1], key=lambda x: p2.index(x)) + p1[c1:]


def cross_PMX(p1, p2, d, W):
    S = len(p1)
    if d == 0:
        d = max(1, int(round(S * 0.3)))
    if d > S:
        return list(p1)
    p1 = p1[:]
    p2 = p2[:]
    r = ints(W).randint(0, S - d)
    c1 = p1[r:r + d]
    c2 = p2[r:r + d]
    pnew = p1[:]
    pnew[r:r + d] = c2
    candidate_indices = list(range(r)) + list(range(r + d, S))   # ascending (see module doc)
    while c1 != []:
        n = c1[0]
        while c2[0] in c1:
            if n == c2[0]:
                break
            link_idx = c1.index(c2[0])
            link = c2[link_idx]
            del c2[link_idx]
            del c1[link_idx]
            c2[0] = link
        if n != c2[0]:
            if n in c2:
                c2[c2.index(n)] = c2[0]
            else:
                for idx in candidate_indices:
                    if pnew[idx] == c2[0]:
                        pnew[idx] = c1[0]
                        candidate_indices.remove(idx)
                        break
        del c1[0]
        del c2[0]
    return pnew


def cross_CX(p1, p2, d, W):
    S = len(p1)
    p = p1[:]
    s = ints(W).randint(0, S - 1)
    i = s
    indices = set()
    while len(indices) < S:
        indices.add(i)
        val = p1[i]
        i = p2.index(val)
        while i in indices:
            if i == s:
                break
            i = p2[i + 1:].index(val) + i + 1
        if i == s:
            break
    for j in indices:
        p[j] = p2[j]
    return p


def cross_OX1(p1, p2, d, W):
    S = len(p1)
    if d == 0:
        d = max(1, int(round(S * 0.3)))
    if d > S:
        return list(p1)
    c1 = p1[:]
    r = ints(W).randint(0, S - d)
    for i in p2[r:r + d]:
        c1.remove(i)
    return c1[:r] + p2[r:r + d] + c1[r:]


def cross_OX3(p1, p2, d, W):
    S = len(p1)
    if d == 0:
        d = max(1, int(round(S * 0.3)))
    if d > S:
        return list(p1)
    c1 = p1[:]
    R = ints(W)
    r1 = R.randint(0, S - d)
    r2 = R.randint(0, S - d)
    for i in p2[r2:r2 + d]:
        c1.remove(i)
    return c1[:r1] + p2[r2:r2 + d] + c1[r1:]


CROSS = {X_OX1: cross_OX1, X_OX3: cross_OX3, X_PX: cross_PX, X_CX: cross_CX, X_PMX: cross_PMX}


def cross(xop, p1, p2, d, W):
    if xop == X_NONE:
        return list(p1)
    return CROSS[xop](list(p1), list(p2), d, W)


def swarm_d(S, strength=0.3):
    """op3_cross: dd = int(round(self.size * strength))"""
    return int(round(S * strength))


def randomized(base, W):
    x = list(base)
    shuffle(x, W)
    return x


def identity(S):
    return list(range(S))
