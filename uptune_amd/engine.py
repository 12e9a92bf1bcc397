"""BatchEngine: the Python face of libuthot.so.

Owns one ut_ctx (one GPU, one HIP stream = torch's current stream on that
device, so library kernels and torch.distributed collectives are ordered on
the same queue).  All large arrays are torch tensors resident in HBM; only
their data pointers cross the C ABI.
"""
from __future__ import annotations

import ctypes as C
from typing import Any, Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import _lib as L
from .manipulator import SpaceSpec, compile_space, to_descs


def _ptr(t: Optional[torch.Tensor]):
    return None if t is None else C.c_void_p(t.data_ptr())


def digests_to_hex(d: torch.Tensor | np.ndarray) -> List[str]:
    """[n][8] big-endian uint32 words (as int32/uint32) -> hexdigest strings"""
    a = d.cpu().numpy() if isinstance(d, torch.Tensor) else np.asarray(d)
    a = a.view(np.uint32).astype(">u4")
    return [row.tobytes().hex() for row in a]


def hex_to_digests(hexes: Sequence[str]) -> np.ndarray:
    """hexdigest strings -> [n][8] uint32 (big-endian word values)"""
    if not hexes:
        return np.zeros((0, 8), dtype=np.uint32)
    raw = np.frombuffer(b"".join(bytes.fromhex(h) for h in hexes), dtype=">u4").reshape(-1, 8)
    return raw.astype(np.uint32)


def _xop(name) -> int:
    if name is None:
        return L.UT_X_NONE
    if isinstance(name, int):
        return name
    if name not in L.CROSSOVERS:
        raise ValueError(f"unknown permutation crossover {name!r} (one of {sorted(L.CROSSOVERS)})")
    return L.CROSSOVERS[name]


class BatchEngine:
    """One device context over one search space."""

    def __init__(self, space, device: int = 0, seed: int = 0, py2_layout: bool = False):
        self.lib = L.lib()
        if not torch.cuda.is_available():
            raise L.UthotError("uptune_amd.BatchEngine needs a ROCm GPU (torch.cuda.is_available() is False)")
        self.device = torch.device("cuda", device)
        self.seed = int(seed)
        self.spec: SpaceSpec = space if isinstance(space, SpaceSpec) else compile_space(space)
        ctx = C.c_void_p()
        torch.cuda.set_device(self.device)
        L.check(None, self.lib.ut_ctx_create(device, self.seed, C.byref(ctx)), "ut_ctx_create")
        self.ctx = ctx
        self._bind_stream()
        descs, keep = to_descs(self.spec)
        L.check(self.ctx, self.lib.ut_space_define(self.ctx, self.spec.P, descs, 1 if py2_layout else 0),
                "ut_space_define")
        del keep
        self.npop = 0
        self.slot = 0
        self._slot_npop: Dict[int, int] = {}
        self.forest = None

    # -- plumbing ----------------------------------------------------------
    def _bind_stream(self):
        s = torch.cuda.current_stream(self.device)
        self._stream = s
        L.check(self.ctx, self.lib.ut_set_stream(self.ctx, C.c_void_p(s.cuda_stream)), "ut_set_stream")

    def close(self):
        if getattr(self, "ctx", None):
            self.lib.ut_ctx_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __deepcopy__(self, memo):
        # techniques are deepcopied per SearchDriver (driver.py:75); a device
        # context is never copied -- the copy re-creates it lazily
        return None

    def sync(self):
        L.check(self.ctx, self.lib.ut_sync(self.ctx), "ut_sync")

    def device_bytes(self) -> int:
        """ut_device_bytes: device memory libuthot holds on this engine's GPU in
        this process (every context; one rank per GPU makes it the rank's footprint)"""
        b = C.c_int64()
        L.check(self.ctx, self.lib.ut_device_bytes(self.device.index, C.byref(b)), "ut_device_bytes")
        return int(b.value)

    def space_info(self) -> Tuple[int, int, int]:
        a, b, c = C.c_int64(), C.c_int64(), C.c_int32()
        L.check(self.ctx, self.lib.ut_space_info(self.ctx, C.byref(a), C.byref(b), C.byref(c)), "ut_space_info")
        return a.value, b.value, c.value

    def _empty(self, *shape, dtype=torch.float64) -> torch.Tensor:
        return torch.empty(*shape, dtype=dtype, device=self.device)

    # -- population --------------------------------------------------------
    def population_init(self, npop: int, round_: int = 0):
        L.check(self.ctx, self.lib.ut_population_init(self.ctx, int(npop), int(round_)), "ut_population_init")
        self.npop = int(npop)

    def population_set(self, values: torch.Tensor):
        values = values.to(self.device, torch.float64).contiguous()
        n = values.shape[1]
        L.check(self.ctx, self.lib.ut_population_set(self.ctx, n, _ptr(values), n), "ut_population_set")
        self.npop = n

    def population_select(self, slot: int):
        """ut_population_select: later population / PSO calls use slot `slot`"""
        if slot == self.slot:
            return
        L.check(self.ctx, self.lib.ut_population_select(self.ctx, int(slot)), "ut_population_select")
        self._slot_npop[self.slot] = self.npop
        self.slot = int(slot)
        self.npop = self._slot_npop.get(self.slot, 0)

    def population_get(self) -> torch.Tensor:
        out = self._empty(self.spec.ncols, self.npop)
        L.check(self.ctx, self.lib.ut_population_get(self.ctx, _ptr(out), self.npop), "ut_population_get")
        return out

    def population_replace(self, trial: torch.Tensor, idx: torch.Tensor):
        trial = trial.contiguous()
        idx = idx.to(self.device, torch.int64).contiguous()
        L.check(self.ctx, self.lib.ut_population_replace(self.ctx, _ptr(trial), trial.shape[1], _ptr(idx),
                                                         idx.numel()), "ut_population_replace")

    # -- proposal ----------------------------------------------------------
    def _de_params(self, cr, n_cross, best, information_sharing):
        """ut_de_params + the device best row it points to (kept alive by the caller)"""
        b = self._row(best)
        p = L.DeParams(cr=float(cr), n_cross=int(n_cross), information_sharing=int(information_sharing),
                       best=None if b is None else b.data_ptr())
        return p, b

    def propose_de(self, m: int, round_: int = 0, cand_base: int = 0, cr: float = 0.2, n_cross: int = 1,
                   out: Optional[torch.Tensor] = None, best=None, information_sharing: int = 1) -> torch.Tensor:
        """DE trials (differentialevolution.py:105-129); `best` = the driver's
        best config as a value row [ncols] (added `information_sharing` times to
        the donor pool, :112-116), None before the first result."""
        if out is None:
            out = self._empty(self.spec.ncols, m)
        p, keep = self._de_params(cr, n_cross, best, information_sharing)
        L.check(self.ctx, self.lib.ut_propose_de(self.ctx, C.byref(p), int(round_), int(cand_base), int(m),
                                                 _ptr(out), out.stride(0)), "ut_propose_de")
        del keep
        return out

    def pso_reset(self):
        L.check(self.ctx, self.lib.ut_pso_reset(self.ctx), "ut_pso_reset")

    def _row(self, r):
        if r is None:
            return None
        if isinstance(r, torch.Tensor):
            return r.to(self.device, torch.float64).contiguous()
        # through pinned memory, asynchronously on the engine's stream (the
        # library's stream, _bind_stream): a pageable copy would wait for every
        # kernel already queued (the fit, the previous stages) before returning
        h = torch.from_numpy(np.ascontiguousarray(r, dtype=np.float64)).pin_memory()
        with torch.cuda.stream(self._stream):
            return h.to(self.device, non_blocking=True)

    def propose_pso(self, gbest, m: int, round_: int = 0, cand_base: int = 0, omega: float = 0.5,
                    phi_l: float = 0.5, phi_g: float = 0.5, sigma: float = 0.2, alias_pbest: bool = True,
                    enum_mode: int = 0, crossover: str = "op3_cross_OX1"):
        """HybridParticle.move for particles (cand_base + i) % npop (pso.py:70-77);
        `crossover` is PSO(crossover=...) for permutation params (pso.py:80-84)."""
        gb = self._row(gbest)
        x = self._empty(self.spec.ncols, m)
        v = self._empty(self.spec.ncols, m)
        a = L.PsoParams(omega=omega, phi_l=phi_l, phi_g=phi_g, sigma=sigma, alias_pbest=1 if alias_pbest else 0,
                        enum_mode=int(enum_mode), crossover=_xop(crossover))
        L.check(self.ctx, self.lib.ut_propose_pso(self.ctx, C.byref(a), _ptr(gb), int(round_), int(cand_base), int(m),
                                                  _ptr(x), _ptr(v), m), "ut_propose_pso")
        return x, v

    def pso_commit(self, values: torch.Tensor, vel: Optional[torch.Tensor], cand_base: int = 0):
        L.check(self.ctx, self.lib.ut_pso_commit(self.ctx, _ptr(values), _ptr(vel), values.stride(0), int(cand_base),
                                                 values.shape[1]), "ut_pso_commit")

    def propose_ga(self, m: int, parent1=None, parent2=None, round_: int = 0, cand_base: int = 0,
                   mutation_rate: float = 0.1, sigma: float = 0.1, crossover_rate: float = 0.0,
                   crossover_strength: float = 0.0, must_mutate_count: int = 1, normal: bool = False,
                   max_retries: int = 10, op: int = 4, crossover: Optional[str] = None):
        """EvolutionaryTechnique / GGA proposals (evolutionarytechniques.py:29-61,
        globalGA.py:28-48 and :68-76); `crossover` = GA(crossover=...) for permutation
        params (CrossoverMixin, :117-134).  Returns (values [ncols][m], invalid [m])."""
        p1, p2 = self._row(parent1), self._row(parent2)
        out = self._empty(self.spec.ncols, m)
        inv = self._empty(m, dtype=torch.uint8)
        a = L.GaParams(mutation_rate=mutation_rate, sigma=sigma, crossover_rate=crossover_rate,
                       crossover_strength=crossover_strength, must_mutate_count=must_mutate_count,
                       normal=1 if normal else 0, max_retries=max_retries, op=op, crossover=_xop(crossover))
        L.check(self.ctx, self.lib.ut_propose_ga(self.ctx, C.byref(a), _ptr(p1), _ptr(p2), int(round_),
                                                 int(cand_base), int(m), _ptr(out), m, _ptr(inv)), "ut_propose_ga")
        return out, inv

    def encode(self, values: torch.Tensor, m: Optional[int] = None) -> torch.Tensor:
        m = values.shape[1] if m is None else m
        feat = self._empty(self.spec.n_features, m)
        L.check(self.ctx, self.lib.ut_encode_features(self.ctx, _ptr(values), values.stride(0), m, _ptr(feat), m),
                "ut_encode_features")
        return feat

    def features_host(self, cfgs: Sequence[Dict[Any, Any]]) -> np.ndarray:
        """configs -> GP features [n][F] (host f64), encoded on the device"""
        if not len(cfgs):
            return np.zeros((0, self.spec.n_features))
        vals = torch.from_numpy(self.spec.encode_configs(cfgs)).to(self.device)
        return self.encode(vals).T.contiguous().cpu().numpy()

    # -- identity / dedup --------------------------------------------------
    def hash(self, values: torch.Tensor, m: Optional[int] = None) -> torch.Tensor:
        m = values.shape[1] if m is None else m
        out = self._empty(m, 8, dtype=torch.int32)
        L.check(self.ctx, self.lib.ut_hash(self.ctx, _ptr(values), values.stride(0), m, _ptr(out)), "ut_hash")
        return out

    def hash_de(self, values: torch.Tensor, cand_base: int = 0, m: Optional[int] = None) -> torch.Tensor:
        """ut_hash_de: hash_config of DE trials proposed from the selected
        population with this cand_base, reusing the targets' inner digests"""
        m = values.shape[1] if m is None else m
        out = self._empty(m, 8, dtype=torch.int32)
        L.check(self.ctx, self.lib.ut_hash_de(self.ctx, _ptr(values), values.stride(0), m, int(cand_base), _ptr(out)),
                "ut_hash_de")
        return out

    def hash_parent(self, values: torch.Tensor, parent, m: Optional[int] = None) -> torch.Tensor:
        """ut_hash_parent: hash_config of GA / GGA children of `parent` (a value
        row), reusing the parent's inner digests for the unchanged params"""
        m = values.shape[1] if m is None else m
        p = self._row(parent)
        out = self._empty(m, 8, dtype=torch.int32)
        L.check(self.ctx, self.lib.ut_hash_parent(self.ctx, _ptr(values), values.stride(0), m, _ptr(p), _ptr(out)),
                "ut_hash_parent")
        return out

    def hash_configs(self, cfgs: Sequence[Dict[Any, Any]]) -> List[str]:
        vals = torch.from_numpy(self.spec.encode_configs(cfgs)).to(self.device)
        d = self.hash(vals)
        return digests_to_hex(d)

    def history_reset(self, capacity: int = 0):
        L.check(self.ctx, self.lib.ut_history_reset(self.ctx, int(capacity)), "ut_history_reset")

    def history_add(self, digests):
        if isinstance(digests, torch.Tensor):
            d = digests.to(self.device, torch.int32).contiguous()
            L.check(self.ctx, self.lib.ut_history_add(self.ctx, _ptr(d), d.shape[0]), "ut_history_add")
        else:
            arr = np.ascontiguousarray(hex_to_digests(digests) if len(digests) and isinstance(digests[0], str)
                                       else np.asarray(digests, dtype=np.uint32).reshape(-1, 8))
            L.check(self.ctx, self.lib.ut_history_add_host(self.ctx, arr.ctypes.data, arr.shape[0]),
                    "ut_history_add_host")

    def dedup(self, digests: torch.Tensor) -> torch.Tensor:
        m = digests.shape[0]
        out = self._empty(m, dtype=torch.uint8)
        L.check(self.ctx, self.lib.ut_dedup(self.ctx, _ptr(digests), m, _ptr(out)), "ut_dedup")
        return out

    # -- GP ----------------------------------------------------------------
    def gp_set_precision(self, bits):
        """64 (fp64 MFMA, 1e-5 tier), 32 (fp32 MFMA, 1e-3 tier), 16 / "f16x3"
        (variance contraction as three fp16 MFMA products of hi/lo splits, f32
        accumulate: the 1e-3 tier at the fp16 MFMA rate) or 8 / "i8" (the fp64
        tier on the int8 MFMA: six-digit slices, a per-candidate error bound,
        fp64 recompute of the candidates it does not clear); applies to later fits"""
        bits = {"f16x3": 16, "i8": 8}.get(bits, bits)
        L.check(self.ctx, self.lib.ut_gp_set_precision(self.ctx, int(bits)), "ut_gp_set_precision")

    def gp_set_prune_pass(self, bits: int):
        """gp_topk_pruned's bound pass: 32 (default, f32 k* with bounded rounding) or 64 (fp64)"""
        L.check(self.ctx, self.lib.ut_gp_set_prune_pass(self.ctx, int(bits)), "ut_gp_set_prune_pass")

    def gp_set_i8_tol(self, tol: float):
        """precision 8: largest accepted relative variance error (0: recompute all in fp64)"""
        L.check(self.ctx, self.lib.ut_gp_set_i8_tol(self.ctx, float(tol)), "ut_gp_set_i8_tol")

    def gp_i8_stats(self) -> Tuple[int, float]:
        """precision 8: (candidates of the last score recomputed in fp64, -1 = all;
        the fit's error bound E on |L^-1 k* - v^|)"""
        n, e = C.c_int64(), C.c_double()
        L.check(self.ctx, self.lib.ut_gp_i8_stats(self.ctx, C.byref(n), C.byref(e)), "ut_gp_i8_stats")
        return int(n.value), float(e.value)

    def gp_i8_bounds(self) -> Tuple[float, float]:
        """precision 8: the fit's bounds (E on the variance's |L^-1 k* - v^|,
        Emu on the mean from the int8 variance epilogue); 0, 0 otherwise"""
        e, em = C.c_double(), C.c_double()
        L.check(self.ctx, self.lib.ut_gp_i8_bounds(self.ctx, C.byref(e), C.byref(em)), "ut_gp_i8_bounds")
        return float(e.value), float(em.value)

    def gp_fit(self, X: np.ndarray, y: np.ndarray, lengthscale, sigma_f2: float = 1.0, sigma_n2: float = 1e-6,
               jitter: float = 0.0, wait: bool = True):
        """ut_gp_fit (wait=True) or ut_gp_fit_async (wait=False: the fit runs on the
        device beside the next round's proposal/hash stages)"""
        X = np.ascontiguousarray(X, dtype=np.float64)
        y = np.ascontiguousarray(y, dtype=np.float64)
        n, d = X.shape
        ell = np.ascontiguousarray(np.broadcast_to(np.asarray(lengthscale, dtype=np.float64), (d,)))
        h = L.GpHyper(sigma_f2=float(sigma_f2), sigma_n2=float(sigma_n2), jitter=float(jitter),
                      lengthscale_host=ell.ctypes.data)
        fn = self.lib.ut_gp_fit if wait else self.lib.ut_gp_fit_async
        L.check(self.ctx, fn(self.ctx, X.ctypes.data, y.ctypes.data, n, d, C.byref(h)), "ut_gp_fit")

    def gp_join_fit(self):
        """ut_gp_join_fit: later work on the engine's stream waits for the
        in-flight fit on the device (no host wait)"""
        L.check(self.ctx, self.lib.ut_gp_join_fit(self.ctx), "ut_gp_join_fit")

    def gp_fit_ok(self) -> bool:
        """ut_gp_fit_status: waits for the last fit; False = its kernel matrix
        was not positive definite (scores are NaN until a fit succeeds)"""
        ok = C.c_int32()
        L.check(self.ctx, self.lib.ut_gp_fit_status(self.ctx, C.byref(ok)), "ut_gp_fit_status")
        return bool(ok.value)

    def gp_set_fit_append(self, enable: bool):
        """incremental fits when the training set only grows (on by default)"""
        L.check(self.ctx, self.lib.ut_gp_set_fit_append(self.ctx, int(bool(enable))), "ut_gp_set_fit_append")

    def gp_last_fit_kind(self) -> str:
        k = C.c_int32()
        L.check(self.ctx, self.lib.ut_gp_last_fit_kind(self.ctx, C.byref(k)), "ut_gp_last_fit_kind")
        return "append" if k.value == 1 else "refit"

    def gp_kstar_mode(self) -> str:
        """ut_gp_kstar_mode: "categorical" (ENUM / BOOL one-hot blocks as an
        int8 code product beside the fp64 contraction) or "dense" """
        v = C.c_int32()
        L.check(self.ctx, self.lib.ut_gp_kstar_mode(self.ctx, C.byref(v)), "ut_gp_kstar_mode")
        return "categorical" if v.value else "dense"

    def gp_stats(self) -> Tuple[float, float, float]:
        a, b, c = C.c_double(), C.c_double(), C.c_double()
        L.check(self.ctx, self.lib.ut_gp_stats(self.ctx, C.byref(a), C.byref(b), C.byref(c)), "ut_gp_stats")
        return a.value, b.value, c.value

    @staticmethod
    def acq(kind: str = "ei", xi: float = 0.0, kappa: float = 2.0) -> L.Acq:
        return L.Acq(kind=L.UT_ACQ_EI if kind == "ei" else L.UT_ACQ_UCB, xi=float(xi), kappa=float(kappa))

    def gp_score(self, feat: torch.Tensor, m: Optional[int] = None, acq: Optional[L.Acq] = None,
                 dup: Optional[torch.Tensor] = None):
        m = feat.shape[1] if m is None else m
        acq = acq or self.acq()
        mu, var, score = self._empty(m), self._empty(m), self._empty(m)
        L.check(self.ctx, self.lib.ut_gp_score(self.ctx, _ptr(feat), feat.stride(0), m, C.byref(acq), _ptr(dup),
                                               _ptr(mu), _ptr(var), _ptr(score)), "ut_gp_score")
        return mu, var, score

    def gp_score_values(self, values: torch.Tensor, m: Optional[int] = None, acq: Optional[L.Acq] = None,
                        dup: Optional[torch.Tensor] = None):
        """ut_gp_score_values: gp_score(encode(values)) with the encoding fused
        into the K* operand pass (no feature matrix)"""
        m = values.shape[1] if m is None else m
        acq = acq or self.acq()
        mu, var, score = self._empty(m), self._empty(m), self._empty(m)
        L.check(self.ctx, self.lib.ut_gp_score_values(self.ctx, _ptr(values), values.stride(0), m, C.byref(acq),
                                                      _ptr(dup), _ptr(mu), _ptr(var), _ptr(score)),
                "ut_gp_score_values")
        return mu, var, score

    def gp_topk_pruned(self, feat: torch.Tensor, k: int, m: Optional[int] = None, acq: Optional[L.Acq] = None,
                       dup: Optional[torch.Tensor] = None, cand_base: int = 0, bound_rows: int = 256):
        """ut_gp_topk_pruned: the top-k of the GP score, selection-exact, with the
        full variance GEMM only for candidates whose score bound (first
        `bound_rows` rows of L^-1 k*) reaches the threshold.  -> (idx, score, stats dict)"""
        m = feat.shape[1] if m is None else m
        acq = acq or self.acq()
        idx = self._empty(k, dtype=torch.int64)
        top = self._empty(k)
        st = L.PruneStats()
        L.check(self.ctx, self.lib.ut_gp_topk_pruned(self.ctx, _ptr(feat), feat.stride(0), m, C.byref(acq), _ptr(dup),
                                                     int(cand_base), int(k), int(bound_rows), _ptr(idx), _ptr(top),
                                                     C.byref(st)), "ut_gp_topk_pruned")
        return idx, top, {"survivors": st.survivors, "bound_rows": st.bound_rows, "dense": bool(st.dense),
                          "threshold": st.threshold, "m": m}

    # -- tree-ensemble surrogate ---------------------------------------------
    def forest_set(self, model):
        """load a tree ensemble (sklearn regressor, XGBoost JSON or forest.Forest)"""
        from .forest import as_forest
        f = as_forest(model)
        nodes = np.ascontiguousarray(f.nodes)
        roots = np.ascontiguousarray(f.roots, dtype=np.int32)
        L.check(self.ctx, self.lib.ut_forest_set(self.ctx, f.n_trees, roots.ctypes.data, nodes.size,
                                                 nodes.ctypes.data, int(f.rule), float(f.base), float(f.scale),
                                                 float(f.div)), "ut_forest_set")
        self.forest = f

    def forest_predict(self, feat: torch.Tensor, m: Optional[int] = None, dup: Optional[torch.Tensor] = None,
                       sign: float = -1.0):
        """-> (pred [m], score [m] = sign * pred, -inf on duplicates)"""
        m = feat.shape[1] if m is None else m
        pred, score = self._empty(m), self._empty(m)
        L.check(self.ctx, self.lib.ut_forest_predict(self.ctx, _ptr(feat), feat.stride(0), m, feat.shape[0],
                                                     _ptr(dup), float(sign), _ptr(pred), _ptr(score)),
                "ut_forest_predict")
        return pred, score

    # -- selection ---------------------------------------------------------
    def topk(self, score: torch.Tensor, k: int, dup: Optional[torch.Tensor] = None, cand_base: int = 0):
        idx = self._empty(k, dtype=torch.int64)
        top = self._empty(k)
        L.check(self.ctx, self.lib.ut_topk(self.ctx, _ptr(score), _ptr(dup), score.numel(), int(cand_base), int(k),
                                           _ptr(idx), _ptr(top)), "ut_topk")
        return idx, top

    # -- whole round -------------------------------------------------------
    def score_round_de(self, m: int, k: int, round_: int = 0, cand_base: int = 0, cr: float = 0.2,
                       n_cross: int = 1, acq: Optional[L.Acq] = None, want_values: bool = True, best=None,
                       information_sharing: int = 1):
        de, keep = self._de_params(cr, n_cross, best, information_sharing)  # noqa: F841 (keeps best alive)
        acq = acq or self.acq()
        idx = self._empty(k, dtype=torch.int64)
        top = self._empty(k)
        dig = self._empty(k, 8, dtype=torch.int32)
        vals = self._empty(self.spec.ncols, k) if want_values else None
        out = L.RoundOut(topk_idx=idx.data_ptr(), topk_score=top.data_ptr(), topk_digest=dig.data_ptr(),
                         topk_values=vals.data_ptr() if vals is not None else None)
        L.check(self.ctx, self.lib.ut_score_round_de(self.ctx, C.byref(de), C.byref(acq), int(round_),
                                                     int(cand_base), int(m), int(k), C.byref(out)),
                "ut_score_round_de")
        return idx, top, dig, vals

    def score_round_ga(self, m: int, k: int, parent1=None, parent2=None, round_: int = 0, cand_base: int = 0,
                       mutation_rate: float = 0.1, sigma: float = 0.1, crossover_rate: float = 0.0,
                       crossover_strength: float = 0.0, must_mutate_count: int = 1, normal: bool = False,
                       max_retries: int = 10, op: int = 4, crossover: Optional[str] = None,
                       acq: Optional[L.Acq] = None, want_values: bool = True):
        """ut_score_round_ga: propose_ga -> hash_parent + dedup (side stream) beside
        encode + GP posterior -> top-k; -> (idx, top, digests, values)"""
        p1, p2 = self._row(parent1), self._row(parent2)
        a = L.GaParams(mutation_rate=mutation_rate, sigma=sigma, crossover_rate=crossover_rate,
                       crossover_strength=crossover_strength, must_mutate_count=must_mutate_count,
                       normal=1 if normal else 0, max_retries=max_retries, op=op, crossover=_xop(crossover))
        acq = acq or self.acq()
        idx = self._empty(k, dtype=torch.int64)
        top = self._empty(k)
        dig = self._empty(k, 8, dtype=torch.int32)
        vals = self._empty(self.spec.ncols, k) if want_values else None
        out = L.RoundOut(topk_idx=idx.data_ptr(), topk_score=top.data_ptr(), topk_digest=dig.data_ptr(),
                         topk_values=vals.data_ptr() if vals is not None else None)
        L.check(self.ctx, self.lib.ut_score_round_ga(self.ctx, C.byref(a), _ptr(p1), _ptr(p2), C.byref(acq),
                                                     int(round_), int(cand_base), int(m), int(k), C.byref(out)),
                "ut_score_round_ga")
        return idx, top, dig, vals

    def score_round_de_pruned(self, m: int, k: int, round_: int = 0, cand_base: int = 0, cr: float = 0.2,
                              n_cross: int = 1, acq: Optional[L.Acq] = None, want_values: bool = True, best=None,
                              information_sharing: int = 1, bound_rows: int = 256):
        """score_round_de with ut_gp_topk_pruned's selection-exact pruning;
        -> (idx, top, digests, values, stats dict)"""
        de, keep = self._de_params(cr, n_cross, best, information_sharing)  # noqa: F841
        acq = acq or self.acq()
        idx = self._empty(k, dtype=torch.int64)
        top = self._empty(k)
        dig = self._empty(k, 8, dtype=torch.int32)
        vals = self._empty(self.spec.ncols, k) if want_values else None
        out = L.RoundOut(topk_idx=idx.data_ptr(), topk_score=top.data_ptr(), topk_digest=dig.data_ptr(),
                         topk_values=vals.data_ptr() if vals is not None else None)
        st = L.PruneStats()
        L.check(self.ctx, self.lib.ut_score_round_de_pruned(self.ctx, C.byref(de), C.byref(acq), int(round_),
                                                            int(cand_base), int(m), int(k), int(bound_rows),
                                                            C.byref(out), C.byref(st)), "ut_score_round_de_pruned")
        return idx, top, dig, vals, {"survivors": st.survivors, "bound_rows": st.bound_rows, "dense": bool(st.dense),
                                     "threshold": st.threshold, "m": m}

    def round_buffers(self):
        ptrs = [C.c_void_p() for _ in range(7)]
        ld = C.c_int64()
        L.check(self.ctx, self.lib.ut_round_buffers(self.ctx, *[C.byref(p) for p in ptrs], C.byref(ld)),
                "ut_round_buffers")
        return [p.value for p in ptrs], ld.value

    def set_timing(self, on: bool):
        L.check(self.ctx, self.lib.ut_set_timing(self.ctx, 1 if on else 0), "ut_set_timing")

    def stage_time(self, stage: str) -> float:
        v = C.c_double()
        L.check(self.ctx, self.lib.ut_stage_time(self.ctx, stage.encode(), C.byref(v)), "ut_stage_time")
        return v.value

    def decode(self, values: torch.Tensor) -> List[Dict[Any, Any]]:
        return self.spec.decode_values(values.detach().cpu().numpy())


_DEFAULT: Dict[int, BatchEngine] = {}


def default_engine(manipulator) -> BatchEngine:
    dev = torch.cuda.current_device() if torch.cuda.is_available() else 0   # this rank's GPU
    key = (id(manipulator), dev)
    eng = _DEFAULT.get(key)
    if eng is None:
        eng = BatchEngine(manipulator, device=dev)
        _DEFAULT[key] = eng
    return eng
