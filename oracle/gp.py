"""fp64 GP surrogate + acquisition -- the build's own specification
("GP spec for a7").  The reference has no GP, Cholesky,
EI or UCB code, so this oracle is NOT pinned by the reference;
it is pinned by tests/golden/gp_*.npz generated from this file.

  us = u / ell                      (ARD length scales)
  K  = sf2 exp(-0.5 |xs_i - xs_j|^2) + (sn2 + jitter) I
  ys = (y - mean(y)) / std(y)       (ddof = 0; std 0 -> 1)
  L  = chol(K);  alpha = K^-1 ys;   f_best = min(ys)
  k* = sf2 exp(-0.5 max(|us|^2 + |xs|^2 - 2 us.xs, 0))
  mu = k*.alpha;  var = max(sf2 - |L^-1 k*|^2, 0)
  EI  = I Phi(z) + sigma phi(z),  I = f_best - mu - xi, z = I / sigma  (sigma == 0: max(I, 0))
  UCB = kappa sigma - mu
"""
import numpy as np
from scipy.linalg import solve_triangular
from scipy.special import erfc


def sqdist(A, B):
    na = np.sum(A * A, axis=1)[:, None]
    nb = np.sum(B * B, axis=1)[None, :]
    d2 = na + nb - 2.0 * (A @ B.T)
    return np.maximum(d2, 0.0)


class GP:
    def __init__(self, X, y, lengthscale, sigma_f2=1.0, sigma_n2=1e-6, jitter=0.0):
        X = np.asarray(X, dtype=np.float64)
        y = np.asarray(y, dtype=np.float64)
        self.inv_ell = 1.0 / np.broadcast_to(np.asarray(lengthscale, dtype=np.float64), (X.shape[1],))
        self.sf2 = float(sigma_f2)
        self.Xs = X * self.inv_ell
        self.mean = float(np.mean(y))
        sd = float(np.sqrt(np.mean((y - self.mean) ** 2)))
        self.std = sd if sd > 0.0 else 1.0
        self.ys = (y - self.mean) / self.std
        self.f_best = float(np.min(self.ys))
        K = self.sf2 * np.exp(-0.5 * sqdist(self.Xs, self.Xs))
        K[np.diag_indices_from(K)] += sigma_n2 + jitter
        self.L = np.linalg.cholesky(K)
        self.alpha = solve_triangular(self.L.T, solve_triangular(self.L, self.ys, lower=True), lower=False)

    def posterior(self, U):
        """U: [m][d] features -> mu, var (standardised units)"""
        Us = np.asarray(U, dtype=np.float64) * self.inv_ell
        Ks = self.sf2 * np.exp(-0.5 * sqdist(Us, self.Xs))
        mu = Ks @ self.alpha
        V = solve_triangular(self.L, Ks.T, lower=True)
        var = np.maximum(self.sf2 - np.sum(V * V, axis=0), 0.0)
        return mu, var


def acquisition(mu, var, f_best, kind="ei", xi=0.0, kappa=2.0):
    sigma = np.sqrt(var)
    if kind == "ucb":
        return kappa * sigma - mu
    I = f_best - mu - xi
    with np.errstate(divide="ignore", invalid="ignore"):
        z = np.where(sigma > 0.0, I / np.where(sigma > 0.0, sigma, 1.0), 0.0)
        Phi = 0.5 * erfc(-z / np.sqrt(2.0))
        phi = np.exp(-0.5 * z * z) / np.sqrt(2.0 * np.pi)
        ei = I * Phi + sigma * phi
    return np.where(sigma > 0.0, ei, np.maximum(I, 0.0))
