"""TEST / MEASUREMENT INFRASTRUCTURE: the batch CPU baseline "B1" of
SURVEY.md §8(d)(ii) -- the C2 round (DE-Alt + hash_config + dedup + GP-EI +
top-k) vectorised over candidates on every host core: C++/OpenMP for DE,
SHA-256 and the dedup set (oracle/cpu_batch.cpp, built by build() into
oracle/_build/libcpubatch.so), NumPy/SciPy BLAS for the GP posterior.  Used by
bench.py's cpu_baseline leg and pinned to the per-candidate oracle by
tests/test_cpu_baseline.py; never imported by uptune_amd/.
"""
import ctypes as C
import os
import subprocess
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "cpu_batch.cpp")
LIB = os.path.join(HERE, "_build", "libcpubatch.so")
CORE = os.path.join(os.path.dirname(HERE), "uptune_amd", "csrc", "ut_core.h")


def build(force=False):
    """g++ -O3 -fopenmp (no -march: the GPU box's host CPU may differ)"""
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    newest = max(os.path.getmtime(SRC), os.path.getmtime(CORE))
    if force or not os.path.exists(LIB) or os.path.getmtime(LIB) < newest:
        subprocess.check_call(["g++", "-O3", "-std=c++17", "-fopenmp", "-ffp-contract=off", "-shared", "-fPIC",
                               "-Wno-deprecated-declarations", SRC,
                               "-o", LIB + ".tmp", "-lcrypto"])
        os.replace(LIB + ".tmp", LIB)
    return LIB


_lib = None


if __name__ == "__main__":
    print(build(force=True))


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = C.CDLL(LIB)
        P = C.c_void_p
        L.cpub_de_hash_float.argtypes = [C.c_int32, P, P, P, C.c_char_p, P, P, C.c_int64, C.c_uint64, C.c_uint32,
                                         C.c_int64, C.c_int64, C.c_double, C.c_int32, P, P]
        L.cpub_de_hash_float.restype = C.c_int
        L.cpub_dedup.argtypes = [P, C.c_int64, P, C.c_int64, P]
        L.cpub_dedup.restype = C.c_int64
        _lib = L
    return _lib


def de_hash_float(space, pop, seed, round_, cand_base, m, cr, n_cross=1):
    """(trial [P][m], digests [m][32] uint8) for a FLOAT-only space"""
    P = len(space)
    lo = np.array([float(p.lo) for p in space])
    hi = np.array([float(p.hi) for p in space])
    order = np.array(sorted(range(P), key=lambda i: space[i].name), dtype=np.int32)
    nb = [str(p.name).encode() for p in space]
    names = b"".join(nb)
    off = np.concatenate([[0], np.cumsum([len(b) for b in nb])]).astype(np.int32)
    pop = np.ascontiguousarray(pop, dtype=np.float64)
    trial = np.empty((P, m))
    dig = np.empty((m, 32), dtype=np.uint8)
    rc = lib().cpub_de_hash_float(P, lo.ctypes.data, hi.ctypes.data, order.ctypes.data, names, off.ctypes.data,
                                  pop.ctypes.data, pop.shape[1], seed, round_, cand_base, m, cr, n_cross,
                                  trial.ctypes.data, dig.ctypes.data)
    if rc != 0:
        raise ValueError("cpub_de_hash_float: bad arguments")
    return trial, dig


def dedup(dig, hist=None):
    hist = np.zeros((0, 32), dtype=np.uint8) if hist is None else np.ascontiguousarray(hist, dtype=np.uint8)
    dup = np.empty(dig.shape[0], dtype=np.uint8)
    lib().cpub_dedup(np.ascontiguousarray(dig).ctypes.data, dig.shape[0], hist.ctypes.data, hist.shape[0],
                     dup.ctypes.data)
    return dup


def topk(score, k):
    """sorted(range(m), key=lambda i: (-s[i], i))[:k] with -inf/NaN excluded, vectorised"""
    s = np.where(np.isnan(score), -np.inf, score)
    kk = min(k, s.size)
    part = np.argpartition(-s, kk - 1)[:kk] if kk < s.size else np.arange(s.size)
    thr = s[part].min()
    cand = np.flatnonzero(s >= thr)                       # every tie of the k-th score
    o = np.lexsort((cand, -s[cand]))[:kk]
    sel = cand[o]
    return sel[np.isfinite(s[sel])]


class BatchPosterior:
    """the oracle GP's posterior restructured for many candidates on many
    cores, as the device does it: L^-1 once per fit (n^3/3), then per chunk
    of candidates K* (GEMM + exp), mu = K* alpha, V = K* L^-T (GEMM) and
    var = sf2 - |V|^2; chunks run on a thread pool (NumPy releases the GIL;
    BLAS single-threaded per chunk).  Same arithmetic as oracle/gp.py up to
    rounding (pinned by tests/test_cpu_baseline.py)."""

    def __init__(self, gp, threads, chunk=8192):
        from scipy.linalg import solve_triangular
        self.gp, self.threads, self.chunk = gp, threads, chunk
        self.LinvT = np.ascontiguousarray(solve_triangular(gp.L, np.eye(gp.L.shape[0]), lower=True).T)
        self.xn = np.sum(gp.Xs * gp.Xs, axis=1)

    def _part(self, U):
        g = self.gp
        Us = U * g.inv_ell
        d2 = np.sum(Us * Us, axis=1)[:, None] + self.xn[None, :] - 2.0 * (Us @ g.Xs.T)
        Ks = g.sf2 * np.exp(-0.5 * np.maximum(d2, 0.0))
        V = Ks @ self.LinvT
        return Ks @ g.alpha, np.maximum(g.sf2 - np.sum(V * V, axis=1), 0.0)

    def posterior(self, U):
        from concurrent.futures import ThreadPoolExecutor

        from threadpoolctl import threadpool_limits
        # at least one chunk per thread (a 256-thread pool on 2^18 candidates
        # in 8192-row chunks kept 32 threads busy)
        ch = max(256, min(self.chunk, -(-U.shape[0] // self.threads)))
        parts = [U[i:i + ch] for i in range(0, U.shape[0], ch)]
        with threadpool_limits(limits=1), ThreadPoolExecutor(self.threads) as ex:
            out = list(ex.map(self._part, parts))
        return np.concatenate([o[0] for o in out]), np.concatenate([o[1] for o in out])


def c2_round(space, pop, gp, seed, round_, m, k, hist=None, cr=0.2, threads=None):
    """one C2 round on the host: DE + hash + dedup (C++/OpenMP) -> features ->
    GP posterior + EI (BLAS, chunks on `threads` cores) -> top-k"""
    from . import gp as ogp
    trial, dig = de_hash_float(space, pop, seed, round_, 0, m, cr, 1)
    dup = dedup(dig, hist)
    lo = np.array([float(p.lo) for p in space])[:, None]
    hi = np.array([float(p.hi) for p in space])[:, None]
    feat = (trial - lo) / (hi - lo)                        # FLOAT unit encoding (get_unit_value)
    bp = gp if isinstance(gp, BatchPosterior) else BatchPosterior(gp, threads or os.cpu_count())
    mu, var = bp.posterior(np.ascontiguousarray(feat.T))
    ei = ogp.acquisition(mu, var, bp.gp.f_best)
    ei = np.where(dup != 0, -np.inf, ei)
    return topk(ei, k), trial, dig, dup, ei


def b1_baseline(m_sample, n, d, k, seed=1, threads=None):
    """candidates/s of the C2 round on `threads` host cores (OpenMP + BLAS)"""
    from threadpoolctl import threadpool_info, threadpool_limits

    from . import de as ode
    from . import gp as ogp
    from .space import FLOAT, Param
    threads = threads or int(os.environ.get("OMP_NUM_THREADS", "0")) or os.cpu_count()
    space = [Param(i, FLOAT, -1000.0, 1000.0) for i in range(d)]
    rng = np.random.default_rng(seed + 100)
    X = rng.uniform(size=(n, d))
    xs = X * 2000.0 - 1000.0
    y = np.sum(100.0 * (xs[:, 1:] - xs[:, :-1] ** 2) ** 2 + (xs[:, :-1] - 1.0) ** 2, axis=1)
    pop = ode.population_init(space, m_sample, seed)
    lib()
    # OpenMP (DE + hash) and the posterior's chunk pool on every thread; the
    # fit's BLAS calls on no more threads than OpenBLAS started with (its
    # buffers are sized then: asked for more -- 32 or 256 where the box's
    # OMP_NUM_THREADS is 16 -- it crashes in solve_triangular)
    blas_threads = min([threads] + [i["num_threads"] for i in threadpool_info() if i.get("user_api") == "blas"])
    with threadpool_limits(limits=threads, user_api="openmp"), \
            threadpool_limits(limits=blas_threads, user_api="blas"):
        c2_round(space, pop[:, :4096], ogp.GP(X, y, lengthscale=0.2), seed, 0, 4096, k, threads=threads)  # warm-up
        t0 = time.perf_counter()
        gp = BatchPosterior(ogp.GP(X, y, lengthscale=0.2, sigma_f2=1.0, sigma_n2=1e-6), threads)
        c2_round(space, pop, gp, seed, 1, m_sample, k, threads=threads)
        dt = time.perf_counter() - t0
    return {"value": m_sample / dt, "unit": "candidates/s", "cores": threads, "kind": "port",
            "sample": f"B1 batch port: oracle/cpu_batch.cpp (C++/OpenMP DE-Alt + repr + OpenSSL SHA-256 "
                      f"hash_config + dedup set) + NumPy/SciPy BLAS GP fit n={n} (L^-1 once) + chunked K*/L^-1 K* "
                      f"GEMM posterior + EI + top-{k}, {m_sample} R64 candidates, {threads} threads "
                      f"(the fit's BLAS on {blas_threads}), {dt:.2f} s"}
