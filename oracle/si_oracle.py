"""StableIdentification CPU restatement — TEST INFRASTRUCTURE ONLY (never imported by the product).

Problem (``src/StableIdentification/coordinator.py:34-152``): minimise over
M = SkewSymmetric(d) x SPD(d) x SPD(d) (pymanopt Product, ``:38-44``)

    f(J, R, Q) = tr(E E^T) / N,   E = XP - (I + h A) X,   A = (J - R) Q        (``:92-98``)

subject to box constraints on entries of A (``:102-152``, rows of ``constset.csv``):
  type 0/1 (one box, two constraints):  -A_rc + ls <= 0  and  A_rc - rs <= 0
  type 2   (two box, one constraint):   -(A_rc - c)^2 + k^2 <= 0
X / XP = the noisy trajectories ``noisyX_<i>.csv`` (``is_X_noisy: True``, Xset 1..5,
``config_simulation.yaml:10-12``) without their last / first column, stacked side by side.

Manifold formulas restate pymanopt (not in this container, **parity unpinned** at that boundary,
SURVEY.md §8c and Appendix B); autograd derivatives are restated in closed form.  Points and
tangent vectors are (3, d, d) arrays [J, R, Q]: elementwise arithmetic is what pymanopt's
``_ProductTangentVector`` does, so the control flow of ``riptrm_oracle.RIPTRMOracle`` runs
unchanged.

Two back-ends with the interface of ``riptrm_oracle.NonnegPCA*``:
  SIStructured  per-constraint loops exactly as RIPTRM.py:475-571 and utils.py:33-203 wire them
                (each constraint's Riemannian gradient / Hessian, metric inner products via solve)
  SIVectorized  the Lagrangian aggregated through dL/dA (the op-for-op twin of the HIP kernel):
                sum_i y_i rhess g_i = e2rh(sum_i y_i egrad g_i, sum_i y_i ehess g_i) (linearity),
                <rgrad g_i, v>_x = Dg_i(x)[v] = (dg_i/dA) : dA(v) for tangent v.
"""
from __future__ import annotations

import copy
import os
from typing import List, Optional, Sequence

import numpy as np

from . import riptrm_oracle as RO


def multisym(a):
    return 0.5 * (a + a.T)


def multiskew(a):
    return 0.5 * (a - a.T)


# ---------------------------------------------------------------------------------------------
# pymanopt manifolds (restated)
# ---------------------------------------------------------------------------------------------
class SkewSymmetric:
    """pymanopt.manifolds.SkewSymmetric(d): Euclidean subspace of skew matrices."""

    def __init__(self, d: int):
        self.d = d
        self.dim = d * (d - 1) // 2
        self.typical_dist = np.sqrt(self.dim)

    def inner_product(self, x, u, v):
        return float(np.tensordot(u, v, axes=u.ndim))

    def norm(self, x, u):
        return np.linalg.norm(u)

    def projection(self, x, u):
        return multiskew(u)

    def euclidean_to_riemannian_gradient(self, x, g):
        return self.projection(x, g)

    def euclidean_to_riemannian_hessian(self, x, g, h, u):
        return self.projection(x, h)

    def retraction(self, x, u):
        return x + u

    def dist(self, a, b):
        return np.linalg.norm(a - b)


class SymmetricPositiveDefinite:
    """pymanopt.manifolds.SymmetricPositiveDefinite(d), affine-invariant metric."""

    def __init__(self, d: int):
        self.d = d
        self.dim = d * (d + 1) // 2
        self.typical_dist = np.sqrt(self.dim)

    def inner_product(self, x, u, v):
        pu = np.linalg.solve(x, u)
        pv = pu if u is v else np.linalg.solve(x, v)
        return float(np.tensordot(pu, pv.T, axes=u.ndim))

    def norm(self, x, u):
        return np.sqrt(self.inner_product(x, u, u))

    def projection(self, x, u):
        return multisym(u)

    def euclidean_to_riemannian_gradient(self, x, g):
        return x @ multisym(g) @ x

    def euclidean_to_riemannian_hessian(self, x, g, h, u):
        return x @ multisym(h) @ x + multisym(u @ multisym(g) @ x)

    def retraction(self, x, u):
        return multisym(x + u + u @ np.linalg.solve(x, u) / 2)

    def dist(self, a, b):
        c = np.linalg.cholesky(a)
        ci = np.linalg.inv(c)
        w = np.linalg.eigvalsh(multisym(ci @ b @ ci.T))
        return np.linalg.norm(np.log(w))        # ||logm(c^-1 b c^-T)||_F


class ProductSkewSPDSPD:
    """pymanopt Product([SkewSymmetric(d), SPD(d), SPD(d)]) on (3, d, d) arrays."""

    def __init__(self, d: int):
        self.d = d
        self.parts = [SkewSymmetric(d), SymmetricPositiveDefinite(d), SymmetricPositiveDefinite(d)]
        self.dim = sum(m.dim for m in self.parts)
        self.typical_dist = np.sqrt(sum(m.typical_dist ** 2 for m in self.parts))

    def inner_product(self, x, u, v):
        return sum(m.inner_product(x[k], u[k], v[k]) for k, m in enumerate(self.parts))

    def norm(self, x, u):
        return np.sqrt(self.inner_product(x, u, u))

    def projection(self, x, u):
        return np.stack([m.projection(x[k], u[k]) for k, m in enumerate(self.parts)])

    to_tangent_space = projection

    def zero_vector(self, x):
        return np.zeros((3, self.d, self.d))

    def euclidean_to_riemannian_gradient(self, x, g):
        return np.stack([m.euclidean_to_riemannian_gradient(x[k], g[k]) for k, m in enumerate(self.parts)])

    def euclidean_to_riemannian_hessian(self, x, g, h, u):
        return np.stack([m.euclidean_to_riemannian_hessian(x[k], g[k], h[k], u[k])
                         for k, m in enumerate(self.parts)])

    def retraction(self, x, u):
        return np.stack([m.retraction(x[k], u[k]) for k, m in enumerate(self.parts)])

    def dist(self, a, b):
        return np.sqrt(sum(m.dist(a[k], b[k]) ** 2 for k, m in enumerate(self.parts)))


# ---------------------------------------------------------------------------------------------
# Data
# ---------------------------------------------------------------------------------------------
class SIData:
    """X, XP, h, the constraint list and d (coordinator.py:49-152)."""

    def __init__(self, X, XP, h, constset):
        self.X = np.asarray(X, dtype=np.float64)
        self.XP = np.asarray(XP, dtype=np.float64)
        self.h = float(h)
        self.d = self.X.shape[0]
        self.N = self.X.shape[1]
        cons = []   # (kind, r, c, p0, p1): kind 0 = -A_rc + ls, 1 = A_rc - rs, 2 = -(A_rc-c)^2 + k^2
        for row in np.atleast_2d(np.asarray(constset, dtype=np.float64)):
            t, r, c = row[0], int(row[1]), int(row[2])
            if t == 0 or t == 1:
                cons.append((0, r, c, float(row[3]), 0.0))
                cons.append((1, r, c, float(row[4]), 0.0))
            elif t == 2:
                cons.append((2, r, c, float(row[3]), float(row[4]) ** 2))
            else:
                raise ValueError("Invalid constraint type")
        self.cons = cons
        self.m = len(cons)

    @staticmethod
    def load(dataset_path: str, Xset: Sequence[int] = (1, 2, 3, 4, 5), h: float = 0.02, noisy: bool = True):
        X = XP = None
        for i in Xset:
            Xo = np.loadtxt(os.path.join(dataset_path, f"{'noisyX' if noisy else 'X'}_{i}.csv"))
            n = Xo.shape[1]
            Xc, XPc = Xo[:, :n - 1], Xo[:, 1:n]
            X = Xc if X is None else np.hstack((X, Xc))
            XP = XPc if XP is None else np.hstack((XP, XPc))
        return SIData(X, XP, h, np.loadtxt(os.path.join(dataset_path, "constset.csv")))


def load_start(dataset_path: str, pt: str):
    """initial point [J, R, Q] (coordinator.py:170-179) and multipliers (:159-163)."""
    x0 = np.stack([np.loadtxt(os.path.join(dataset_path, f"init{c}_{pt}.csv")) for c in "JRQ"])
    y0 = np.atleast_1d(np.loadtxt(os.path.join(dataset_path, "initineqLagmult.csv")))
    return x0, y0


def synthetic_instance(d: int, seed: int, starts: int = 1, **kw):
    """A StableIdentification instance of block size d by the reference's dataset recipe: the
    product's restatement si.synthetic_problem (src/StableIdentification/generator.py:18-134, its one
    deviation documented there), wrapped as SIData.  Returns (SIData, [(x0, y0), ...])."""
    import si
    X, XP, h, constset, st = si.synthetic_problem(d, seed, starts=starts, **kw)
    return SIData(X, XP, h, constset), st


def si_manvio(x):
    """src/StableIdentification/simulator.py:11-32 (the PD test prints and returns inf)."""
    J, R, Q = x[0], x[1], x[2]
    mv = np.linalg.norm(J + J.T) + np.linalg.norm(R - R.T) + np.linalg.norm(Q - Q.T)
    if not np.all(np.linalg.eigvalsh(R) > 0) or not np.all(np.linalg.eigvalsh(Q) > 0):
        mv = np.inf
    return mv


# ---------------------------------------------------------------------------------------------
# Closed-form derivatives (autograd restated)
# ---------------------------------------------------------------------------------------------
def _A(x):
    return (x[0] - x[1]) @ x[2]


def _dA(x, v):
    return (v[0] - v[1]) @ x[2] + (x[0] - x[1]) @ v[2]


def _chain(x, G):
    """egrad of phi(A(J,R,Q)) from G = dphi/dA."""
    gq = G @ x[2].T
    return np.stack([gq, -gq, (x[0] - x[1]).T @ G])


def _chain_hess(x, G, dG, v):
    """ehess of phi(A(J,R,Q)) along v from G = dphi/dA and dG = D(dphi/dA)[dA(v)]."""
    t = dG @ x[2].T + G @ v[2].T
    return np.stack([t, -t, (v[0] - v[1]).T @ G + (x[0] - x[1]).T @ dG])


class _SIBase:
    gpu_pass_accounting = False

    def __init__(self, data: SIData):
        self.D = data
        self.d = data.d
        self.manifold = ProductSkewSPDSPD(data.d)
        self.matvecs = 0

    # f and its A-derivatives
    def cost(self, x):
        D = self.D
        A = _A(x)
        At = np.eye(self.d) + D.h * A
        E = D.XP - At @ D.X
        return np.trace(E @ E.T) / D.N

    def _GA_cost(self, x):
        D = self.D
        E = D.XP - (np.eye(self.d) + D.h * _A(x)) @ D.X
        return -(2.0 * D.h / D.N) * (E @ D.X.T)

    def _dGA_cost(self, x, dA):
        D = self.D
        return (2.0 * D.h * D.h / D.N) * (dA @ (D.X @ D.X.T))

    def ineq_values(self, x):
        A = _A(x)
        out = np.empty(self.D.m)
        for i, (k, r, c, p0, p1) in enumerate(self.D.cons):
            a = A[r, c]
            out[i] = (-a + p0) if k == 0 else ((a - p0) if k == 1 else (-(a - p0) ** 2 + p1))
        return out

    def _wA(self, x):
        """dg_i/dA = w_i E_{r_i c_i}."""
        A = _A(x)
        w = np.empty(self.D.m)
        for i, (k, r, c, p0, p1) in enumerate(self.D.cons):
            w[i] = -1.0 if k == 0 else (1.0 if k == 1 else -2.0 * (A[r, c] - p0))
        return w

    def slack(self, x):
        return -self.ineq_values(x)

    def tangent_basis(self, x):
        from .trs_oracle import si_tangent_basis
        return si_tangent_basis(x)

    def maxmeanviolations(self, x):
        mx, mean = 0, 0
        for g in self.ineq_values(x):
            v = max(g, 0)
            mx = max(mx, v)
            mean += v
        if self.D.m > 0:
            mean = mean / self.D.m
        return mx, mean


class SIStructured(_SIBase):
    """Per-constraint wiring of utils.NonlinearProblem + RIPTRM.py:475-571 (False branches)."""

    def __init__(self, data: SIData):
        super().__init__(data)
        M = self.manifold
        self.euclidean_gradient = lambda x: _chain(x, self._GA_cost(x))
        self.euclidean_hessian = lambda x, v: _chain_hess(x, self._GA_cost(x), self._dGA_cost(x, _dA(x, v)), v)
        self.riemannian_gradient = lambda x: M.euclidean_to_riemannian_gradient(x, self.euclidean_gradient(x))
        self.riemannian_hessian = lambda x, v: M.euclidean_to_riemannian_hessian(
            x, self.euclidean_gradient(x), self.euclidean_hessian(x, v), v)

        def mk(i):
            k, r, c, p0, p1 = data.cons[i]

            def g(x):
                a = _A(x)[r, c]
                return (-a + p0) if k == 0 else ((a - p0) if k == 1 else (-(a - p0) ** 2 + p1))

            def GA(x):
                G = np.zeros((self.d, self.d))
                G[r, c] = -1.0 if k == 0 else (1.0 if k == 1 else -2.0 * (_A(x)[r, c] - p0))
                return G

            def dGA(x, v):
                G = np.zeros((self.d, self.d))
                if k == 2:
                    G[r, c] = -2.0 * _dA(x, v)[r, c]
                return G

            eg = lambda x: _chain(x, GA(x))
            eh = lambda x, v: _chain_hess(x, GA(x), dGA(x, v), v)
            rg = lambda x: M.euclidean_to_riemannian_gradient(x, eg(x))
            rh = lambda x, v: M.euclidean_to_riemannian_hessian(x, eg(x), eh(x, v), v)
            return g, rg, rh

        cons = [mk(i) for i in range(data.m)]
        self.ineq = [c[0] for c in cons]
        self.ineq_rgrad = [c[1] for c in cons]
        self.ineq_rhess = [c[2] for c in cons]

    def gradlag(self, x, y):
        vec = self.riemannian_gradient(x)
        gv = [-grad(x) for grad in self.ineq_rgrad]
        for i in range(len(y)):
            vec = vec - y[i] * gv[i]
        return vec

    def hesslag(self, x, y, dx):
        vec = self.riemannian_hessian(x, dx)
        hv = [-h(x, dx) for h in self.ineq_rhess]
        for i in range(len(y)):
            vec = vec - y[i] * hv[i]
        return vec

    def Gx(self, x, v):
        gv = [-grad(x) for grad in self.ineq_rgrad]
        vec = self.manifold.zero_vector(x)
        for idx in range(len(gv)):
            vec = vec + v[idx] * gv[idx]
        return vec

    def Gxaj(self, x, dx):
        gv = [-grad(x) for grad in self.ineq_rgrad]
        return np.array([self.manifold.inner_product(x, g, dx) for g in gv])

    def begin_inner(self, x, y, mu):
        cx = self.cost(x)
        s = self.slack(x)
        gradcostx = self.riemannian_gradient(x)
        Hw = lambda dx: self.hesslag(x, y, dx) + self.Gx(x, (y * self.Gxaj(x, dx)) / s)
        c = gradcostx - self.Gx(x, mu / s)
        return cx, s, Hw, c

    def dy(self, x, y, s, mu, dx):
        return -y + mu * (1 / s) - y * self.Gxaj(x, dx) / s

    def residual(self, x, y, manviofun):
        M = self.manifold
        vec = self.riemannian_gradient(x)
        for i in range(self.D.m):
            vec = vec + y[i] * self.ineq_rgrad[i](x)
        gradnorm = M.norm(x, vec)
        sq_compl = sum((y[i] * self.ineq[i](x)) ** 2 for i in range(self.D.m))
        sq_nonneg = sum(max(-v, 0) ** 2 for v in y)
        sq_ineq = sum(max(self.ineq[i](x), 0) ** 2 for i in range(self.D.m))
        manvio = manviofun(x)
        residual = np.sqrt(gradnorm ** 2 + sq_compl + sq_nonneg + sq_ineq + 0 + manvio ** 2)
        return residual, gradnorm, np.sqrt(sq_compl), np.sqrt(sq_nonneg), manvio


class SIVectorized(_SIBase):
    """Lagrangian aggregated through dL/dA: the twin of the HIP kernel (riptrm_si.hip)."""

    def _scatter(self, coef):
        G = np.zeros((self.d, self.d))
        for i, (k, r, c, p0, p1) in enumerate(self.D.cons):
            G[r, c] += coef[i]
        return G

    def riemannian_gradient(self, x):
        return self.manifold.euclidean_to_riemannian_gradient(x, _chain(x, self._GA_cost(x)))

    def gradlag(self, x, y):
        G = self._GA_cost(x) + self._scatter(y * self._wA(x))
        return self.manifold.euclidean_to_riemannian_gradient(x, _chain(x, G))

    def hesslag(self, x, y, dx):
        dA = _dA(x, dx)
        G = self._GA_cost(x) + self._scatter(y * self._wA(x))
        dG = self._dGA_cost(x, dA)
        for i, (k, r, c, p0, p1) in enumerate(self.D.cons):
            if k == 2:
                dG[r, c] += y[i] * (-2.0 * dA[r, c])
        return self.manifold.euclidean_to_riemannian_hessian(x, _chain(x, G), _chain_hess(x, G, dG, dx), dx)

    def Gxaj(self, x, dx):
        dA = _dA(x, dx)
        w = self._wA(x)
        return np.array([-w[i] * dA[r, c] for i, (k, r, c, p0, p1) in enumerate(self.D.cons)])

    def Gx(self, x, v):
        G = self._scatter(-(np.asarray(v) * self._wA(x)))
        return self.manifold.euclidean_to_riemannian_gradient(x, _chain(x, G))

    def begin_inner(self, x, y, mu):
        cx = self.cost(x)
        s = self.slack(x)
        c = self.riemannian_gradient(x) - self.Gx(x, mu / s)
        Hw = lambda dx: self.hesslag(x, y, dx) + self.Gx(x, (y * self.Gxaj(x, dx)) / s)
        return cx, s, Hw, c

    def dy(self, x, y, s, mu, dx):
        return -y + mu * (1 / s) - y * self.Gxaj(x, dx) / s

    def residual(self, x, y, manviofun):
        M = self.manifold
        G = self._GA_cost(x) + self._scatter(y * self._wA(x))
        gradnorm = M.norm(x, M.euclidean_to_riemannian_gradient(x, _chain(x, G)))
        g = self.ineq_values(x)
        sq_compl = float(np.sum((y * g) ** 2))
        sq_nonneg = float(np.sum(np.maximum(-y, 0) ** 2))
        sq_ineq = float(np.sum(np.maximum(g, 0) ** 2))
        manvio = manviofun(x)
        residual = np.sqrt(gradnorm ** 2 + sq_compl + sq_nonneg + sq_ineq + 0 + manvio ** 2)
        return residual, gradnorm, np.sqrt(sq_compl), np.sqrt(sq_nonneg), manvio


def solve(data: SIData, x0, y0, option=None, structured=False, clock=None) -> RO.OracleResult:
    P = SIStructured(data) if structured else SIVectorized(data)
    kw = {} if clock is None else {"clock": clock}
    opt = {"manviofun": si_manvio}
    opt.update(option or {})
    return RO.RIPTRMOracle(opt, **kw).run(P, np.asarray(x0, dtype=np.float64), np.asarray(y0, dtype=np.float64))
