"""Test infrastructure: a CPU stand-in for uptune_amd.engine.BatchEngine built
on the oracle (oracle/ is the checker, never the product).  It implements the
engine methods the technique layer calls, with the same arguments and the
same results the device gives (the GPU parity tests prove device == oracle),
so the plugin plumbing -- SharedModel, GpuBatchTechnique, the reference-side
binding -- runs end to end in the CPU suite.  Never used by uptune_amd."""
import numpy as np
import torch

from _spaces import oracle_space
from oracle import de as ode
from oracle import ga as oga
from oracle import gp as ogp
from oracle import hashing as oh
from oracle import perm as opm
from oracle import pso as opso
from oracle import select as osel
from oracle.space import features, row_values
from uptune_amd.manipulator import compile_space


class OracleEngine:
    def __init__(self, manipulator, device=0, seed=0):
        self.spec = compile_space(manipulator)
        self.space = oracle_space(manipulator)
        self.seed = int(seed)
        self.device = torch.device("cpu")
        self.slot = 0
        self.npop = 0
        self._slots = {}
        self._hist = set()
        self.gp = None
        self.gp_ok = False
        self.forest = None
        self.calls = {"hash": 0, "gp_fit": 0, "gp_score": 0}

    # -- population slots ---------------------------------------------------
    def _state(self):
        return self._slots.setdefault(self.slot, {"pop": None, "vel": None, "best": None})

    def population_select(self, slot):
        self._state()["npop"] = self.npop
        self.slot = int(slot)
        self.npop = self._state().get("npop", 0)

    def population_init(self, npop, round_=0):
        self._state()["pop"] = ode.population_init(self.space, int(npop), self.seed, round_)
        self.npop = int(npop)

    def population_get(self):
        return torch.from_numpy(self._state()["pop"].copy())

    def population_replace(self, trial, idx):
        st = self._state()
        for j, i in enumerate(idx.tolist()):
            st["pop"][:, i] = trial[:, j].numpy()

    def pso_reset(self):
        st = self._state()
        st["vel"] = np.zeros_like(st["pop"])
        st["best"] = st["pop"].copy()

    # -- proposals ----------------------------------------------------------
    def propose_de(self, m, round_=0, cand_base=0, cr=0.2, n_cross=1, best=None, information_sharing=1):
        best = None if best is None else np.asarray(best, dtype=np.float64)
        return torch.from_numpy(ode.propose_de_vec(self.space, self._state()["pop"], self.seed, round_, cand_base, m,
                                                   cr, n_cross, best=best, information_sharing=information_sharing))

    def propose_pso(self, gbest, m, round_=0, cand_base=0, omega=0.5, phi_l=0.5, phi_g=0.5, sigma=0.2,
                    alias_pbest=True, enum_mode=0, crossover="op3_cross_OX1"):
        st = self._state()
        gb = gbest.numpy() if isinstance(gbest, torch.Tensor) else np.asarray(gbest, dtype=np.float64)
        pb = st["pop"] if alias_pbest else st["best"]
        x, v = opso.propose_pso_vec(self.space, st["pop"], st["vel"], pb, gb, self.seed, round_, cand_base, m,
                                    omega, phi_l, phi_g, sigma, enum_mode, opm.XNAMES.get(crossover, opm.X_OX1))
        return torch.from_numpy(x), torch.from_numpy(v)

    def pso_commit(self, x, v, cand_base=0):
        st = self._state()
        n = x.shape[1]
        st["pop"][:, cand_base:cand_base + n] = x.numpy()
        st["vel"][:, cand_base:cand_base + n] = v.numpy()

    def propose_ga(self, m, parent1=None, parent2=None, round_=0, cand_base=0, crossover=None, **kw):
        p1 = None if parent1 is None else np.asarray(parent1, dtype=np.float64)
        p2 = None if parent2 is None else np.asarray(parent2, dtype=np.float64)
        xop = opm.XNAMES.get(crossover, opm.X_NONE) if crossover else opm.X_NONE
        vals, inv = oga.propose_ga_vec(self.space, p1, p2, self.seed, round_, cand_base, m, crossover=xop, **kw)
        return torch.from_numpy(vals), torch.from_numpy(inv.astype(np.uint8))

    # -- identity -----------------------------------------------------------
    def hash(self, vals):
        self.calls["hash"] += 1
        v = vals.numpy()
        hx = [oh.hash_config(self.space, row_values(self.space, v, j)) for j in range(v.shape[1])]
        raw = np.frombuffer(b"".join(bytes.fromhex(h) for h in hx), dtype=">u4").reshape(-1, 8)
        return torch.from_numpy(raw.astype(np.uint32).view(np.int32).copy())

    def hash_de(self, vals, cand_base=0):
        return self.hash(vals)

    def hash_configs(self, cfgs):
        from uptune_amd.engine import digests_to_hex
        return digests_to_hex(self.hash(torch.from_numpy(self.spec.encode_configs(cfgs))))

    def history_reset(self, capacity=0):
        self._hist = set()

    def history_add(self, digests):
        self._hist.update(digests)

    def dedup(self, dig):
        from uptune_amd.engine import digests_to_hex
        return torch.tensor(osel.dedup(digests_to_hex(dig), self._hist), dtype=torch.uint8)

    # -- surrogate ----------------------------------------------------------
    def encode(self, vals, m=None):
        return torch.from_numpy(features(self.space, vals.numpy()))

    def features_host(self, cfgs):
        if not len(cfgs):
            return np.zeros((0, self.spec.n_features))
        return features(self.space, self.spec.encode_configs(cfgs)).T.copy()

    def gp_set_precision(self, bits):
        pass

    def gp_fit(self, X, y, lengthscale, sigma_f2=1.0, sigma_n2=1e-6, jitter=0.0, wait=True):
        """as ut_gp_fit_async: a kernel matrix that is not positive definite
        does not raise; scores are NaN until a fit succeeds (gp_fit_ok)"""
        self.calls["gp_fit"] += 1
        self.calls.setdefault("jitter", []).append(jitter)
        try:
            self.gp = ogp.GP(X, y, lengthscale=lengthscale, sigma_f2=sigma_f2, sigma_n2=sigma_n2, jitter=jitter)
            self.gp_ok = True
        except np.linalg.LinAlgError:
            self.gp_ok = False

    def gp_fit_ok(self):
        return self.gp_ok

    @staticmethod
    def acq(kind="ei", xi=0.0, kappa=2.0):
        return (kind, xi, kappa)

    def gp_score(self, feat, m=None, acq=None, dup=None):
        self.calls["gp_score"] += 1
        kind, xi, kappa = acq or ("ei", 0.0, 2.0)
        if not self.gp_ok:
            nan = torch.full((feat.shape[1],), float("nan"), dtype=torch.float64)
            return nan, nan.clone(), nan.clone()
        mu, var = self.gp.posterior(feat.numpy().T)
        sc = ogp.acquisition(mu, var, self.gp.f_best, kind=kind, xi=xi, kappa=kappa)
        if dup is not None:
            sc = np.where(dup.numpy() != 0, -np.inf, sc)
        return torch.from_numpy(mu), torch.from_numpy(var), torch.from_numpy(sc)

    def gp_score_values(self, values, m=None, acq=None, dup=None):
        return self.gp_score(self.encode(values), m, acq, dup)

    def topk(self, score, k, dup=None, cand_base=0):
        s = score.numpy().tolist()
        d = None if dup is None else dup.numpy().tolist()
        sel = osel.topk(s, k, dup=d, cand_base=cand_base)
        top = [s[i - cand_base] if i >= 0 else -np.inf for i in sel]
        return torch.tensor(sel, dtype=torch.int64), torch.tensor(top, dtype=torch.float64)

    def decode(self, rows):
        return self.spec.decode_values(rows.numpy())
