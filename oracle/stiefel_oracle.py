"""Stiefel(n, p) manifold operations (pymanopt 2.x restated) — TEST INFRASTRUCTURE ONLY.

SURVEY.md §8a row A14: the Stiefel manifold is required by north_star / BASELINE configs[4] but
does not occur in the reference (its problems live on Sphere, Grassmann and Product(Skew, SPD,
SPD)), and pymanopt is not in this container: **parity unpinned** — these are the published
pymanopt formulas, checked by identities (tests/test_stiefel_oracle.py) and used as the checker
of the HIP kernels (csrc/riptrm_stiefel.hip).

  inner(X, U, V)      = tensordot(U, V)  (= tr(U^T V))
  projection(X, U)    = U - X sym(X^T U)
  retraction(X, U)    = qf(X + U): Q of the QR factorisation with diag(R) > 0
  e2rg(X, G)          = projection(X, G)
  e2rh(X, G, H, U)    = projection(X, H - U sym(X^T G))
  dim = n p - p (p + 1) / 2,  typical_dist = sqrt(p)
"""
from __future__ import annotations

import numpy as np


def multisym(a):
    return 0.5 * (a + np.swapaxes(a, -1, -2))


class Stiefel:
    def __init__(self, n: int, p: int):
        if p > n:
            raise ValueError("need p <= n")
        self.n, self.p = n, p
        self.dim = n * p - p * (p + 1) // 2
        self.typical_dist = np.sqrt(p)

    def inner_product(self, X, U, V):
        return float(np.tensordot(U, V, axes=U.ndim))

    def norm(self, X, U):
        return np.linalg.norm(U)

    def projection(self, X, U):
        return U - X @ multisym(X.T @ U)

    to_tangent_space = projection

    def euclidean_to_riemannian_gradient(self, X, G):
        return self.projection(X, G)

    def euclidean_to_riemannian_hessian(self, X, G, H, U):
        return self.projection(X, H - U @ multisym(X.T @ G))

    def retraction(self, X, U):
        q, r = np.linalg.qr(X + U)
        return q * np.sign(np.sign(np.diag(r)) + 0.5)   # qf: flip columns so that diag(R) > 0

    def zero_vector(self, X):
        return np.zeros_like(X)

    def random_point(self, rs):
        q, r = np.linalg.qr(rs.randn(self.n, self.p))
        return q * np.sign(np.sign(np.diag(r)) + 0.5)

    def random_tangent_vector(self, X, rs):
        u = self.projection(X, rs.randn(self.n, self.p))
        return u / np.linalg.norm(u)
