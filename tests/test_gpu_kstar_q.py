"""Precision-8 K* as the distance contraction on the int8 MFMA (gp_kq.hip,
the default) against k_gp_kstar<int8_t> on the fp64 MFMA (UT_KSTAR_Q=0): both
are the fp64 tier (the int8 contraction's digit rounding is below the fp64
contraction's own, gp_kq.hip), so every candidate's mean and variance agree to
1e-9 relative (1e-10 absolute) and the dense rounds select the same
candidates, at the padded sizes 1024 / 2048 (sf2 far from 1 too: the round-5
fault case, npad 2048 and sf2 1e-3).  A categorical fit keeps the fp64-MFMA K*
(bit-identical with and without UT_KSTAR_Q).  Both are held to
oracle/gp.py by test_gpu_i8.py / test_gpu_parity.py."""
import ctypes
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from oracle import de as ode  # noqa: E402
from oracle import gp as ogp  # noqa: E402
from oracle.space import BOOL, ENUM, FLOAT, INT, Param, features  # noqa: E402

pytestmark = pytest.mark.gpu

from _spaces import to_manip  # noqa: E402

SPACES = {
    "r64": [Param(f"x{j}", FLOAT, -1000.0, 1000.0) for j in range(64)],
    "cat": [Param("x", FLOAT, -5.0, 5.0), Param("n", INT, 1, 64), Param("flag", BOOL),
            Param("mode", ENUM, options=["a", "b", "c", 4]), Param("y", FLOAT, 0.0, 1.0),
            Param("sel", ENUM, options=[str(i) for i in range(9)]), Param("big", INT, -100000, 2000000)],
}


def _d2h(ptr, m):
    hip = ctypes.CDLL("libamdhip64.so")
    out = np.empty(m, dtype=np.float64)
    rc = hip.hipMemcpy(ctypes.c_void_p(out.ctypes.data), ctypes.c_void_p(ptr), ctypes.c_size_t(8 * m), 2)
    assert rc == 0, rc
    return out


def _round(monkeypatch, space, q, n, sf2, ell):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    monkeypatch.setenv("UT_KSTAR_Q", "1" if q else "0")
    from uptune_amd.engine import BatchEngine
    e = BatchEngine(to_manip(space), device=0, seed=5)
    e.gp_set_precision(8)
    npop, m, k = 3000, 20000, 64
    pop = ode.population_init(space, npop, seed=5)
    e.population_set(torch.from_numpy(np.ascontiguousarray(pop)).to("cuda:0"))
    X = features(space, pop[:, :n]).T
    y = np.sum((X - 0.45) ** 2, axis=1)
    e.history_reset(0)
    e.gp_fit(X, y, lengthscale=ell, sigma_f2=sf2, sigma_n2=1e-6 * sf2, jitter=1e-8 * sf2, wait=False)
    idx, top, dig, vals = e.score_round_de(m, k, round_=1, cand_base=0, cr=0.3)
    e.sync()
    (pv, _, _, _, pmu, pvar, psc), ld = e.round_buffers()
    vals = _d2h(pv, ld * len(space)).reshape(len(space), ld)[:, :m]   # (while the engine holds them)
    return (idx.cpu().numpy(), top.cpu().numpy(), _d2h(pmu, m), _d2h(pvar, m), _d2h(psc, m),
            e.gp_kstar_mode(), X, y, vals)


@pytest.mark.parametrize("which", ["r64", "cat"])
@pytest.mark.parametrize("n,sf2,ell", [(1000, 1.0, 2.0), (2000, 1e-3, 0.8)])
def test_kstar_q_equals_fp64_kstar(monkeypatch, which, n, sf2, ell):
    space = SPACES[which]
    a = _round(monkeypatch, space, True, n, sf2, ell)
    b = _round(monkeypatch, space, False, n, sf2, ell)
    assert a[5] == b[5] == ("dense" if which == "r64" else "categorical")
    if which == "cat":
        # categorical fits keep the fp64-MFMA K* (gp.hip gp_score_impl): the same kernels
        for x, y in zip(a[:5], b[:5]):
            np.testing.assert_array_equal(x, y)
        return
    # (the two contractions round differently at ~1e-12 of the operands' scale;
    # the tier's bound on the mean is E_mu ~1e-7, on the variance tau = 2^-20)
    np.testing.assert_allclose(a[2], b[2], rtol=1e-9, atol=1e-10)          # mean
    np.testing.assert_allclose(a[3], b[3], rtol=1e-9, atol=1e-10 * sf2)    # variance
    np.testing.assert_allclose(a[4], b[4], rtol=1e-9, atol=1e-10)          # EI
    # the same selections wherever the scores are apart
    s = np.sort(a[4])[::-1]
    if np.min(np.abs(np.diff(s[:65]))) > 1e-8 * max(abs(s[0]), 1e-300):
        np.testing.assert_array_equal(a[0], b[0])


def test_kstar_q_round_against_oracle(monkeypatch):
    """the int8 K* round's mean / variance of a sample of candidates against
    the oracle's posterior (1e-5, the north star's fp64 tolerance)"""
    space = SPACES["r64"]
    idx, top, mu, var, sc, mode, X, y, vals = _round(monkeypatch, space, True, 1000, 1.0, 2.0)
    pick = np.arange(0, 20000, 97)
    g = ogp.GP(X, y, lengthscale=2.0, sigma_f2=1.0, sigma_n2=1e-6, jitter=1e-8)
    mu_o, var_o = g.posterior(features(space, vals[:, pick]).T)
    np.testing.assert_allclose(mu[pick], mu_o, rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(var[pick], var_o, rtol=1e-5, atol=1e-8)
