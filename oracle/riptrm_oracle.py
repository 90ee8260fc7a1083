"""CPU oracle for the RIPTRM tCG hot path — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
this module, and only as the checker / the timed CPU baseline.  The product path
(``riemannian-interior-point-trust-region-method_amd/``) never imports it and never falls back to it.

What it is
----------
A NumPy fp64 restatement of the reference solver ``RIPTRM`` (``src/solver/RIPTRM.py``) on the
path every shipped config selects (``TRS_solver='tCG'``, ``second_order_stationarity=False``,
``src/NonnegPCA/config_simulation.yaml:20-24``), for the NonnegPCA problem on the sphere
(``src/NonnegPCA/coordinator.py:37-95``).  Two problem back-ends share one control flow:

* ``NonnegPCAStructured`` mirrors the reference's per-constraint plumbing
  (``src/solver/utils.py:33-203`` + ``RIPTRM.py:475-571``): n constraint closures, the
  per-constraint loops of ``Gxfun``/``Gxajfun``/``hessLagrangefun``, the same summation order.
  O(n^2) per Hessian-vector product; used for n <= 200.
* ``NonnegPCAVectorized`` is the closed form with ``S = Z + Z^T`` and the
  same algebra, pass structure and caching that the HIP kernels implement (one S-pass per tCG
  iteration plus one two-right-hand-side pass per trial point).  This is the GPU's op-for-op twin
  and the CPU baseline ("port" kind) timed by ``bench.py``.

Pinning (read this before trusting it)
--------------------------------------
The reference cannot be imported or run in this container (pymanopt/autograd/hydra absent,
``RIPTRM.py:806`` needs Python >= 3.12).  Its derivative math lives in
un-vendored, unpinned pymanopt + autograd; the formulas below restate pymanopt 2.x
(SURVEY.md Appendix B).  The reference holds no golden outputs and no tests.  What pins this
oracle is therefore only:

1. the known answer stored in ``src/NonnegPCA/analyzer.ipynb`` (cell 5 printed output): every
   solver's first log row for ``dataset/NonnegPCA/1`` point ``a`` has KKT residual
   ``4.986888e+00`` (``tests/test_oracle.py::test_initial_residual_known_answer``);
2. the published qualitative result (``analyzer.ipynb`` cell 5 plot): RIPTRM (tCG) on that
   fixture drives the KKT residual to ~1e-14 and stays there
   (``tests/test_oracle.py::test_fixture_run_reaches_published_residual``);
3. internal consistency: the structured and vectorized back-ends agree, derivatives match
   finite differences, tCG invariants hold.

Trajectory-level parity with the reference's own iterates is therefore **partially pinned**
(parity unpinned beyond the two checks above); see DESIGN.md "Oracle and parity".
"""
from __future__ import annotations

import copy
import math
import time
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional

import numpy as np
import scipy.linalg
from scipy.linalg.blas import dsymv as _dsymv

SPACING1 = np.spacing(1)  # RIPTRM.py:660 np.spacing(1)

# tCG stop strings (RIPTRM.py:95,143,145,164,188,190)
TCG_STOPS = ("MAX_INNER_ITER", "NEGATIVE_CURVATURE", "EXCEEDED_TR", "MODEL_INCREASED",
             "REACHED_TARGET_LINEAR", "REACHED_TARGET_SUPERLINEAR")


# ---------------------------------------------------------------------------------------------
# pymanopt 2.x Sphere, restated (call sites RIPTRM.py:44,47,210,735,744,857)
# ---------------------------------------------------------------------------------------------
class Sphere:
    def __init__(self, n: int):
        self.n = int(n)
        self.dim = self.n - 1          # RIPTRM.py:447 maxinner = manifold.dim
        self.typical_dist = math.pi    # RIPTRM.py:857 Delta_bar

    def inner_product(self, x, u, v):
        return np.tensordot(u, v, axes=u.ndim)

    def norm(self, x, v):
        return np.linalg.norm(v)

    def projection(self, x, u):
        return u - self.inner_product(x, x, u) * x

    to_tangent_space = projection

    def zero_vector(self, x):
        return np.zeros_like(x)

    def retraction(self, x, v):
        w = x + v
        return w / np.linalg.norm(w)

    def dist(self, a, b):
        inner = max(min(self.inner_product(a, a, b), 1), -1)
        return np.arccos(inner)

    def euclidean_to_riemannian_gradient(self, x, g):
        return self.projection(x, g)

    def weingarten(self, x, v, normal):
        return -self.inner_product(x, x, normal) * v

    def euclidean_to_riemannian_hessian(self, x, egrad, ehess, v):
        normal = egrad - self.projection(x, egrad)
        return self.projection(x, ehess) + self.weingarten(x, v, normal)


# ---------------------------------------------------------------------------------------------
# Problem back-ends
# ---------------------------------------------------------------------------------------------
def sphere_tangent_basis(x, rs=None):
    """Orthonormal basis of T_x Sphere(n) for Exact_RepMat (RIPTRM.py:436 basisfun).
    rs=None: the columns 1..n-1 of the Householder reflector H = I - tau w w^T, w = x + sign(x_0)
    ||x|| e_0 (what the device uses).  rs = RandomState: the reference's tangentorthobasis
    (utils.py:388-397) — random tangent vectors, Gram-Schmidt in the manifold metric (utils.py:
    375-386).  The subproblem's solution does not depend on the choice."""
    x = np.asarray(x, dtype=np.float64)
    n = len(x)
    if rs is None:
        w = x.copy()
        w[0] += (1.0 if x[0] >= 0 else -1.0) * np.sqrt(x @ x)
        tau = 2.0 / (w @ w)
        return [np.eye(n)[k] - tau * w * w[k] for k in range(1, n)]
    Q = []
    for _ in range(n - 1):
        v = rs.randn(n)
        v = v - (x @ v) * x
        v = v / np.linalg.norm(v)
        for q in Q:
            v = v - (q @ v) * q
        Q.append(v / np.linalg.norm(v))
    return Q


class NonnegPCAStructured:
    """Per-constraint restatement of NonnegPCA + NonlinearProblem + RIPTRM's G/H helpers.

    cost      src/NonnegPCA/coordinator.py:52-54   f(x) = -x^T Z x  (autograd derivatives restated)
    ineq      src/NonnegPCA/coordinator.py:66-75   g_i(x) = -x_i  (egrad -e_i, ehess 0)
    wrappers  src/solver/utils.py:93-173           rgrad_i = P_x(egrad_i); rhess_i = e2rh(...)
    helpers   src/solver/RIPTRM.py:475-571         gradLagrangefun/hessLagrangefun/Gxfun/Gxajfun

    ``lincomb`` / ``embedded`` select the reference's ``do_euclidean_lincomb=True`` /
    ``is_euclidean_embedded=True`` branches (RIPTRM.py:480-482, :514-517, :543-545, :567-568):
    Euclidean linear combinations converted once, and <egrad g_i, dx> in place of <rgrad g_i, dx>.
    On the Sphere both give the same operators as the default branches on tangent vectors (the
    conversions are linear; <-e_i, dx> = <P_x(-e_i), dx> when x^T dx = 0), so they differ from the
    default only by rounding (tests/test_oracle.py::test_euclidean_branch_options_agree).
    """

    def __init__(self, Z: np.ndarray, lincomb: bool = False, embedded: bool = False):
        self.lincomb = bool(lincomb)
        self.embedded = bool(embedded)
        self.Z = np.asarray(Z, dtype=np.float64)
        self.n = self.Z.shape[0]
        self.manifold = Sphere(self.n)
        self.matvecs = 0
        n = self.n
        M = self.manifold

        def cost(x):
            return -x @ self.Z @ x

        def egrad(x):
            self.matvecs += 2
            return ((-x) @ self.Z) + (-(self.Z @ x))

        def ehess(x, v):
            self.matvecs += 2
            return -(self.Z @ v) - (v @ self.Z)

        self.cost = cost
        self.euclidean_gradient = egrad
        self.euclidean_hessian = ehess
        self.riemannian_gradient = lambda x: M.euclidean_to_riemannian_gradient(x, egrad(x))
        self.riemannian_hessian = lambda x, v: M.euclidean_to_riemannian_hessian(x, egrad(x), ehess(x, v), v)

        def mk(i):
            e = np.zeros(n)
            e[i] = -1.0
            g = lambda x: -x[i]
            eg = lambda x: e.copy()
            eh = lambda x, v: np.zeros(n)
            rg = lambda x: M.euclidean_to_riemannian_gradient(x, eg(x))
            rh = lambda x, v: M.euclidean_to_riemannian_hessian(x, eg(x), eh(x, v), v)
            return g, eg, eh, rg, rh

        cons = [mk(i) for i in range(n)]
        self.ineq = [c[0] for c in cons]
        self.ineq_egrad = [c[1] for c in cons]
        self.ineq_ehess = [c[2] for c in cons]
        self.ineq_rgrad = [c[3] for c in cons]
        self.ineq_rhess = [c[4] for c in cons]

    # RIPTRM.py:721 costineqconstvecfun
    def tangent_basis(self, x):
        return sphere_tangent_basis(x)

    def slack(self, x):
        return np.array([-g(x) for g in self.ineq])

    # RIPTRM.py:457-473 egradLagrangefun
    def egradlag(self, x, y):
        vec = self.euclidean_gradient(x)
        ev = [-eg(x) for eg in self.ineq_egrad]
        for i in range(len(y)):
            vec = vec - y[i] * ev[i]
        return vec

    # RIPTRM.py:475-489
    def gradlag(self, x, y):
        if self.lincomb:
            return self.manifold.euclidean_to_riemannian_gradient(x, self.egradlag(x, y))
        vec = self.riemannian_gradient(x)
        gv = [-grad(x) for grad in self.ineq_rgrad]
        for i in range(len(y)):
            vec = vec - y[i] * gv[i]
        return vec

    # RIPTRM.py:491-523
    def hesslag(self, x, y, dx):
        if self.lincomb:   # :514-517
            vec = self.euclidean_hessian(x, dx)
            ehv = [-eh(x, dx) for eh in self.ineq_ehess]
            for i in range(len(y)):
                vec = vec - y[i] * ehv[i]
            return self.manifold.euclidean_to_riemannian_hessian(x, self.egradlag(x, y), vec, dx)
        vec = self.riemannian_hessian(x, dx)
        hv = [-h(x, dx) for h in self.ineq_rhess]
        for i in range(len(y)):
            vec = vec - y[i] * hv[i]
        return vec

    # RIPTRM.py:525-551
    def Gx(self, x, v):
        if self.lincomb:   # :543-545
            ev = [-eg(x) for eg in self.ineq_egrad]
            vec = self.manifold.zero_vector(x)
            for idx in range(len(ev)):
                vec = vec + v[idx] * ev[idx]
            return self.manifold.euclidean_to_riemannian_gradient(x, vec)
        gv = [-grad(x) for grad in self.ineq_rgrad]
        vec = self.manifold.zero_vector(x)
        for idx in range(len(gv)):
            vec = vec + v[idx] * gv[idx]
        return vec

    # RIPTRM.py:553-571
    def Gxaj(self, x, dx):
        if self.embedded:   # :567-568
            ev = [-eg(x) for eg in self.ineq_egrad]
            return np.array([self.manifold.inner_product(x, g, dx) for g in ev])
        gv = [-grad(x) for grad in self.ineq_rgrad]
        return np.array([self.manifold.inner_product(x, g, dx) for g in gv])

    # RIPTRM.py:724-730
    def begin_inner(self, x, y, mu):
        cx = self.cost(x)
        s = self.slack(x)
        gradcostx = self.riemannian_gradient(x)
        Hw = lambda dx: self.hesslag(x, y, dx) + self.Gx(x, (y * self.Gxaj(x, dx)) / s)
        c = gradcostx - self.Gx(x, mu / s)
        return cx, s, Hw, c

    # RIPTRM.py:743
    def dy(self, x, y, s, mu, dx):
        return -y + mu * (1 / s) - y * self.Gxaj(x, dx) / s

    # utils.py:269-340 compute_residual (ineq only, no eq constraints)
    def residual(self, x, y, manviofun):
        M = self.manifold
        vec = self.riemannian_gradient(x)
        for i in range(self.n):
            vec = vec + y[i] * self.ineq_rgrad[i](x)
        gradnorm = M.norm(x, vec)
        sq_grad = gradnorm ** 2
        sq_compl = 0
        for i in range(self.n):
            sq_compl += (y[i] * self.ineq[i](x)) ** 2
        complvio = np.sqrt(sq_compl)
        sq_nonneg = 0
        for v in y:
            sq_nonneg += max(-v, 0) ** 2
        nonnegvio = np.sqrt(sq_nonneg)
        sq_ineq = 0
        for i in range(self.n):
            sq_ineq += max(self.ineq[i](x), 0) ** 2
        manvio = manviofun(x)
        residual = np.sqrt(sq_grad + sq_compl + sq_nonneg + sq_ineq + 0 + manvio ** 2)
        return residual, gradnorm, complvio, nonnegvio, manvio

    # utils.py:237-267
    def maxmeanviolations(self, x):
        mx = 0
        mean = 0
        for i in range(self.n):
            v = max(self.ineq[i](x), 0)
            mx = max(mx, v)
            mean += v
        if self.n > 0:
            mean = mean / self.n
        return mx, mean


class NonnegPCAVectorized:
    """Closed-form NonnegPCA — the op-for-op twin of the HIP kernels.

    S = Z + Z^T.  Per inner step the only dense work is S.v (one pass per tCG iteration) and one
    fused two-right-hand-side pass (S.dx, S.x_new) at the trial point; S.x is cached per iterate.
    Every formula below is the one ``csrc/riptrm_kernels.hip`` evaluates, in the same order.
    """

    def __init__(self, Z: np.ndarray, S: Optional[np.ndarray] = None, symv: bool = True):
        Z = np.asarray(Z, dtype=np.float64)
        self.n = Z.shape[0]
        # Fortran order so BLAS dsymv streams one triangle (half the bytes of dgemv), the CPU
        # analogue of the GPU's symmetric-tile layout
        self.S = np.asfortranarray((Z + Z.T) if S is None else S)
        self.symv = symv
        self.manifold = Sphere(self.n)
        self.matvecs = 0          # S.v products
        self._sx_key = None
        self._sx = None

    def Sv(self, v):
        self.matvecs += 1
        if self.symv:
            return _dsymv(1.0, self.S, v)
        return self.S @ v

    def Sx(self, x):
        if self._sx_key is not x:
            self._sx = self.Sv(x)
            self._sx_key = x
        return self._sx

    def cost(self, x):
        return -0.5 * (x @ self.Sx(x))

    def tangent_basis(self, x):
        return sphere_tangent_basis(x)

    def slack(self, x):
        return x.copy()

    def riemannian_gradient(self, x):
        g = -self.Sx(x)
        return g - (x @ g) * x

    def gradlag(self, x, y):
        g = self.riemannian_gradient(x)
        return g - (y - (y @ x) * x)

    def Gxaj(self, x, v):
        return v - x * (x @ v)

    def Gx(self, x, w):
        return w - (x @ w) * x

    def begin_inner(self, x, y, mu):
        cx = self.cost(x)
        s = self.slack(x)
        gradcostx = self.riemannian_gradient(x)
        xx = x @ x
        coef = (x @ self.Sx(x) + y @ x) * xx

        def Hw(v):
            u = self.Sv(v)
            hf = -u + (x @ u) * x
            q = (y * (v - x * (x @ v))) / s
            return hf + coef * v + (q - (x @ q) * x)

        m = mu / s
        c = gradcostx - (m - (x @ m) * x)
        return cx, s, Hw, c

    def dy(self, x, y, s, mu, dx):
        return -y + mu * (1 / s) - y * (dx - x * (x @ dx)) / s

    def residual(self, x, y, manviofun):
        g = self.gradlag(x, y)
        gradnorm = np.linalg.norm(g)
        compl = y * (-x)
        sq_compl = compl @ compl
        complvio = np.sqrt(sq_compl)
        neg = np.maximum(-y, 0)
        sq_nonneg = neg @ neg
        nonnegvio = np.sqrt(sq_nonneg)
        iv = np.maximum(-x, 0)
        sq_ineq = iv @ iv
        manvio = manviofun(x)
        residual = np.sqrt(gradnorm ** 2 + sq_compl + sq_nonneg + sq_ineq + 0 + manvio ** 2)
        return residual, gradnorm, complvio, nonnegvio, manvio

    def maxmeanviolations(self, x):
        iv = np.maximum(-x, 0)
        mx = max(0.0, iv.max()) if self.n else 0.0
        return mx, (iv.sum() / self.n if self.n else 0.0)


# ---------------------------------------------------------------------------------------------
# RIPTRM control flow (shared by both back-ends)
# ---------------------------------------------------------------------------------------------
def truncated_conjugate_gradient(manifold, hess, x, fgradx, Delta, theta, kappa, mininner, maxinner):
    """Steihaug-Toint tCG, RIPTRM.py:41-216 with use_rand=False, identity preconditioner
    (pymanopt Problem.preconditioner default) and eta0 = 0 (RIPTRM.py:446)."""
    inner = manifold.inner_product
    eta = manifold.zero_vector(x)
    Heta = manifold.zero_vector(x)
    r = fgradx
    e_Pe = 0
    r_r = inner(x, r, r)
    norm_r = np.sqrt(r_r)
    norm_r0 = norm_r
    z = r
    z_r = inner(x, z, r)
    d_Pd = z_r
    delta = -z
    e_Pd = 0
    model_value = 0
    stop = "MAX_INNER_ITER"
    j = 0
    for j in range(int(maxinner)):
        Hdelta = hess(delta)
        d_Hd = inner(x, delta, Hdelta)
        if d_Hd != 0:
            alpha = z_r / d_Hd
            e_Pe_new = e_Pe + 2 * alpha * e_Pd + alpha ** 2 * d_Pd
        else:
            e_Pe_new = e_Pe
        if d_Hd <= 0 or e_Pe_new >= Delta ** 2:
            tau = (-e_Pd + np.sqrt(e_Pd * e_Pd + d_Pd * (Delta ** 2 - e_Pe))) / d_Pd
            eta = eta + tau * delta
            Heta = Heta + tau * Hdelta
            stop = "NEGATIVE_CURVATURE" if d_Hd <= 0 else "EXCEEDED_TR"
            break
        e_Pe = e_Pe_new
        new_eta = eta + alpha * delta
        new_Heta = Heta + alpha * Hdelta
        new_model_value = inner(x, new_eta, fgradx) + 0.5 * inner(x, new_eta, new_Heta)
        if new_model_value >= model_value:
            stop = "MODEL_INCREASED"
            break
        eta = new_eta
        Heta = new_Heta
        model_value = new_model_value
        r = r + alpha * Hdelta
        r_r = inner(x, r, r)
        norm_r = np.sqrt(r_r)
        if j >= mininner and norm_r <= norm_r0 * min(norm_r0 ** theta, kappa):
            stop = "REACHED_TARGET_LINEAR" if kappa < norm_r0 ** theta else "REACHED_TARGET_SUPERLINEAR"
            break
        z = r
        zold_rold = z_r
        z_r = inner(x, z, r)
        beta = z_r / zold_rold
        delta = -z + beta * delta
        delta = manifold.to_tangent_space(x, delta)
        e_Pd = beta * (e_Pd + alpha * d_Pd)
        d_Pd = z_r + beta * beta * d_Pd
    return eta, Heta, j, stop


def default_option() -> Dict[str, Any]:
    """RIPTRM defaults, RIPTRM.py:305-358 (tCG-path keys)."""
    return {
        'maxtime': 240, 'maxiter': 100, 'tolresid': 1e-15,
        'inner_maxiter': None, 'inner_maxtime': None,
        'initial_TR_radius': None, 'minimal_initial_TR_radius': 1e-15, 'maximal_TR_radius': 10,
        'rho': 0.1, 'reduction_regularization': 1e3, 'gamma': 0.25,
        'forcing_function_Lagrangian': lambda mu: max(mu, 1e-14),
        'forcing_function_complementarity': lambda mu: max(1e-3 * mu, 1e-14),
        'forcing_function_second_order': lambda mu: mu,
        'min_barrier_parameter': 1e-15,
        'TRS_solver': 'tCG', 'second_order_stationarity': False, 'TRS_tolhardcase': 1e-8,
        'tCG_theta': 1, 'tCG_kappa': 0.1, 'tCG_mininner': 1,
        'initial_barrier_parameter': 0.1,
        'barrier_parameter_update_r': 0.01, 'barrier_parameter_update_c': 0.5,
        'barrier_parameter_update_b': 0.8, 'do_simple_barrier_parameter_update': True,
        'const_left': 0.5, 'const_right': 1e+20,
        'manviofun': lambda x: 0,
        'save_inner_iteration': True,
    }


def sphere_manvio(x):
    """src/NonnegPCA/simulator.py:12-14 manviofun = ||x|| - 1."""
    return np.linalg.norm(x) - 1


@dataclass
class OracleResult:
    x: np.ndarray
    y: np.ndarray
    log: Dict[str, List[Any]]
    stoppingcriterion: str
    outer_iterations: int
    inner_iterations: int
    tcg_iterations: int
    matvecs: int
    passes: int
    trace: List[Dict[str, Any]] = field(default_factory=list)


class BudgetExceeded(Exception):
    """Raised by RIPTRMOracle when its optional wall-clock deadline passes (bench sampling)."""


class RIPTRMOracle:
    """RIPTRM.run / outer_step / inner_run / inner_step / update_xy_TR_radius restated
    (RIPTRM.py:574-976) for the tCG path.  ``clock`` may be replaced to make time deterministic.
    ``outer_heads[k]`` records the solver time (wall minus excluded evaluation time) at the head
    of outer iteration k, so callers can time a window of outer iterations."""

    def __init__(self, option: Optional[Dict[str, Any]] = None, clock: Callable[[], float] = time.time,
                 deadline: Optional[float] = None):
        opt = default_option()
        if option:
            opt.update(option)
        self.option = opt
        self.clock = clock
        self.log: Dict[str, List[Any]] = {}
        self.excluded_time = 0.0
        self.trace: List[Dict[str, Any]] = []
        self.tcg_total = 0
        self.inner_total = 0
        self.passes = 1        # GPU pass accounting: S.x0 once, then see inner_step
        self.deadline = deadline
        self.outer_heads: Dict[int, float] = {}
        self.inner_durations: List[float] = []   # solver seconds of each completed inner step

    # base_solver.py:58-76
    def add_log(self, it, start_time, ev, status):
        if it == 0 and "iteration" not in self.log:
            self.log["iteration"] = [0]
            self.log["time"] = [0]
            for k, v in ev.items():
                self.log[k] = [v]
            for k, v in status.items():
                self.log[k] = [v]
        else:
            self.log["iteration"].append(it)
            self.log["time"].append(self.clock() - start_time - self.excluded_time)
            for k, v in ev.items():
                self.log[k].append(v)
            for k, v in status.items():
                self.log[k].append(v)

    # utils.py:342-368
    def evaluation(self, P, xPrev, x, y):
        cost = P.cost(x)
        dist = P.manifold.dist(xPrev, x)
        residual, gradnorm, complvio, nonnegvio, manvio = P.residual(x, y, self.option['manviofun'])
        mx, mean = P.maxmeanviolations(x)
        return {"cost": cost, "distance": dist, "residual": residual, "gradnorm": gradnorm,
                "complviolation": complvio, "dualviolation": nonnegvio, "manviolation": manvio,
                "maxviolation": mx, "meanviolation": mean}

    # RIPTRM.py:980-1024
    @staticmethod
    def solver_status(y, mu, save_inner, info=None):
        st = {"mu": mu}
        keys_basic = ("num_inner", "inner_status", "TR_radius")
        for k in keys_basic:
            st[k] = None if info is None else info[k]
        if save_inner:
            for k in ("dxtype", "normdx", "minxfeasi", "minyfeasi", "compl", "mineigvalHw",
                      "ared/pred", "radius_update", "dual_clipping"):
                st[k] = None if info is None else info[k]
        m = float('-inf')
        for v in y:
            m = max(m, abs(v))
        st["maxabsLagmult"] = m
        return st

    @staticmethod
    def initial_inner_info(inner_iteration, TR_radius):
        return {"inner_status": None, "num_inner": inner_iteration, "TR_radius": TR_radius,
                "normdx": None, "dxtype": None, "minxfeasi": None, "minyfeasi": None,
                "compl": None, "mineigvalHw": None, "ared/pred": None, "radius_update": None,
                "dual_clipping": None}

    # RIPTRM.py:574-629 (tCG path; eigen-check skipped)
    def inner_criteria(self, P, xNew, yNew, mu, inner_option):
        sNew = P.slack(xNew)
        out = {}
        out["xfeasi_criterion"] = bool(np.all(sNew > 0))
        out["yfeasi_criterion"] = bool(np.all(yNew > 0))
        normgl = P.manifold.norm(xNew, P.gradlag(xNew, yNew))
        out["normgradLagfun_criterion"] = normgl <= inner_option["stopping_criterion_Lagrangian"]
        compl = np.linalg.norm(yNew * sNew - mu)
        out["complementary_criterion"] = compl <= inner_option["stopping_criterion_complementarity"]
        out["minxfeasi"] = min(sNew)
        out["minyfeasi"] = min(yNew)
        out["compl"] = compl
        out["sNew"] = sNew
        o = self.option
        if o['TRS_solver'] == 'Exact_RepMat' and o['second_order_stationarity']:   # RIPTRM.py:599-617
            from .trs_oracle import selfadj_operator2matrix
            _, _, HwNew, _ = P.begin_inner(xNew, yNew, mu)
            try:
                Hm = selfadj_operator2matrix(P.manifold, xNew, HwNew, P.tangent_basis(xNew))
                mineig = scipy.linalg.eigh(Hm, eigvals_only=True)[0]
            except np.linalg.LinAlgError:
                mineig = np.nan
            out["mineigvalHw"] = mineig
            out["mineigval_criterion"] = bool(mineig >= -o['forcing_function_second_order'](mu))
        return out

    # RIPTRM.py:631-705
    def update_xy_TR_radius(self, P, x, y, sCur, Hw, c, dx, normdx, xNew, yNew, sNew, mu, Delta):
        o = self.option
        M = P.manifold

        def logbarr(xx, ss):
            return P.cost(xx) - mu * np.sum(np.log(ss))

        lb_cur = logbarr(x, sCur)
        lb_new = logbarr(xNew, sNew)
        ared = lb_cur - lb_new
        pred = 0 - 0.5 * M.inner_product(x, Hw(dx), dx) - M.inner_product(x, c, dx)
        red_reg = max(1, abs(lb_cur)) * SPACING1 * o['reduction_regularization']
        ared = ared + red_reg
        pred = pred + red_reg
        out = {"ared/pred": ared / pred}
        if ared < 0.25 * pred:
            out["radius_update"] = "reduced"
            Dn = 0.25 * Delta
        elif ared >= 0.75 * pred and np.abs(normdx - Delta) <= 1e-15:
            out["radius_update"] = "expanded"
            Dn = min(2 * Delta, o['maximal_TR_radius'])
        else:
            out["radius_update"] = "unchanged"
            Dn = Delta
        if ared > o['rho'] * pred:
            out["inner_status"] = "successful"
            xn = copy.deepcopy(xNew)
            I_left = o['const_left'] * np.minimum(np.minimum(y, mu / sNew), 1)
            # RIPTRM.py:682: 3-arg np.maximum writes max(cr, cr/mu) into `out` (y/s terms discarded)
            I_right = np.maximum(o['const_right'], o['const_right'] / mu,
                                 np.maximum(y, o['const_right'] / sNew))
            yc = np.minimum(np.maximum(yNew, I_left), I_right)
            out["dual_clipping"] = not np.array_equal(yNew, yc)
            yn = yc
        else:
            out["inner_status"] = "unsuccessful"
            out["dual_clipping"] = None
            xn, yn = x, y
        return xn, yn, Dn, out

    # RIPTRM.py:707-783
    def inner_step(self, P, x, y, mu, Delta, inner_iteration, inner_option):
        o = self.option
        info = self.initial_inner_info(inner_iteration, Delta)
        M = P.manifold
        cx, s, Hw, c = P.begin_inner(x, y, mu)
        if o['TRS_solver'] == 'Exact_RepMat':   # RIPTRM.py:433-444 (trs_oracle)
            from .trs_oracle import exact_repmat_direction
            dx, _, kind, _ = exact_repmat_direction(M, x, Hw, c, Delta, P.tangent_basis(x), o['TRS_tolhardcase'])
            j, stop = -1, None
            info["dxtype"] = kind
        else:
            dx, _, j, stop = truncated_conjugate_gradient(M, Hw, x, c, Delta, o['tCG_theta'], o['tCG_kappa'],
                                                          o['tCG_mininner'], M.dim)
            info["dxtype"] = f"tCG_{stop}"
        # Hessian-vector products performed inside tCG = j + 1 (loop index at exit)
        self.tcg_total += j + 1
        self.passes += j + 1
        normdx = M.norm(x, dx)
        info["normdx"] = normdx
        dy = P.dy(x, y, s, mu, dx)
        xNew = M.retraction(x, dx)
        yNew = y + dy
        if getattr(P, "gpu_pass_accounting", True) and np.all(xNew > 0):
            self.passes += 1   # GPU: one fused pass computes S.dx (pred) and S.x_new
        cr = self.inner_criteria(P, xNew, yNew, mu, inner_option)
        info["minxfeasi"] = cr["minxfeasi"]
        info["minyfeasi"] = cr["minyfeasi"]
        info["compl"] = cr["compl"]
        info["mineigvalHw"] = cr.get("mineigvalHw")
        rec = {"tcg_iters": j + 1, "tcg_stop": stop, "normdx": normdx, "Delta": Delta, "mu": mu}
        if (cr["xfeasi_criterion"] and cr["yfeasi_criterion"] and cr["normgradLagfun_criterion"]
                and cr["complementary_criterion"] and cr.get("mineigval_criterion", True)):
            info["inner_status"] = "converged"
            rec["status"] = "converged"
            self.trace.append(rec)
            return True, xNew, yNew, Delta, info
        if not cr["xfeasi_criterion"]:
            info["inner_status"] = "primal_infeasible"
            rec["status"] = "primal_infeasible"
            self.trace.append(rec)
            return False, x, y, o['gamma'] * normdx, info
        xn, yn, Dn, up = self.update_xy_TR_radius(P, x, y, s, Hw, c, dx, normdx, xNew, yNew, cr["sNew"], mu, Delta)
        for k in ("ared/pred", "radius_update", "dual_clipping", "inner_status"):
            info[k] = up[k]
        rec.update(status=up["inner_status"], ared_pred=up["ared/pred"], radius_update=up["radius_update"])
        self.trace.append(rec)
        return False, xn, yn, Dn, info

    # RIPTRM.py:785-847
    def inner_run(self, P, outer_iteration, outer_start_time, x0, y0, mu, Delta0, inner_option):
        o = self.option
        x, y, Delta = x0, y0, Delta0
        xPrev = copy.deepcopy(x)
        it = 0
        inner_start = self.clock()
        info = self.initial_inner_info(0, Delta)
        while True:
            it += 1
            if self.deadline is not None and self.clock() > self.deadline:
                raise BudgetExceeded()
            t_step = self.clock()
            exitflag, x, y, Delta, info = self.inner_step(P, x, y, mu, Delta, it, inner_option)
            self.inner_durations.append(self.clock() - t_step)
            self.inner_total += 1
            if o['save_inner_iteration']:
                t0 = self.clock()
                ev = self.evaluation(P, xPrev, x, y)
                st = self.solver_status(y, mu, True, info)
                self.excluded_time += self.clock() - t0
                self.add_log(outer_iteration, outer_start_time, ev, st)
            xPrev = copy.deepcopy(x)
            if o['inner_maxtime'] is None:
                lim = o['maxtime']
                rt = self.clock() - outer_start_time - self.excluded_time
            else:
                lim = o['inner_maxtime']
                rt = self.clock() - inner_start
            if rt >= lim:
                info["inner_status"] = "max-time-exceeded"
                exitflag = True
                x, y, Delta = x0, y0, Delta0
                xPrev = copy.deepcopy(x0)
            if o['inner_maxiter'] is not None and it >= o['inner_maxiter']:
                info["inner_status"] = "max-iter-exceeded"
                exitflag = True
                x, y, Delta = x0, y0, Delta0
                xPrev = copy.deepcopy(x0)
            if exitflag:
                break
        return x, y, Delta, info

    # RIPTRM.py:909-976 (+ outer_preprocess 849-864, outer_step 866-896, base_solver 85-107)
    def run(self, P, x0, y0) -> OracleResult:
        o = self.option
        x = copy.deepcopy(np.asarray(x0, dtype=np.float64))
        y = copy.deepcopy(np.asarray(y0, dtype=np.float64))
        mu = o['initial_barrier_parameter']
        Delta = (P.manifold.typical_dist / 8) if o['initial_TR_radius'] is None else o['initial_TR_radius']
        xPrev = copy.deepcopy(x)
        info = None
        it = 0
        start = self.clock()
        reason = None
        while True:
            t0 = self.clock()
            ev = self.evaluation(P, xPrev, x, y)
            self.excluded_time += self.clock() - t0
            if it == 0 or not o['save_inner_iteration']:
                t0 = self.clock()
                st = self.solver_status(y, mu, o['save_inner_iteration'], info)
                self.excluded_time += self.clock() - t0
                self.add_log(it, start, ev, st)
            residual = ev["residual"]
            xPrev = copy.deepcopy(x)
            rt = self.clock() - start - self.excluded_time
            self.outer_heads[it] = rt
            stop = False
            if rt >= o['maxtime']:
                stop, reason = True, f"Max time exceeded; runtime={rt:.2f} and maxtime={o['maxtime']}"
            elif it >= o['maxiter']:
                stop, reason = True, f"Max iteration count reached; maxiter={o['maxiter']} after {rt:.2f} seconds"
            if residual <= o['tolresid']:
                stop = True
                reason = ("KKT residual tolerance reached; current residual=" + str(residual)
                          + " and tolresid=" + str(o['tolresid']) + f" after {rt:.2f} seconds")
            if stop:
                break
            it += 1
            inner_option = {
                "stopping_criterion_Lagrangian": o['forcing_function_Lagrangian'](mu),
                "stopping_criterion_complementarity": o['forcing_function_complementarity'](mu),
            }
            x, y, Delta, info = self.inner_run(P, it, start, x, y, mu, Delta, inner_option)
            if o['do_simple_barrier_parameter_update']:
                mu = max(o['min_barrier_parameter'],
                         o['barrier_parameter_update_c'] * (mu ** (1 + o['barrier_parameter_update_r'])))
            else:
                mu = max(o['min_barrier_parameter'],
                         min(o['barrier_parameter_update_b'] * mu,
                             o['barrier_parameter_update_c'] * (mu ** (1 + o['barrier_parameter_update_r']))))
            Delta = max(Delta, o['minimal_initial_TR_radius'])
        return OracleResult(x=x, y=y, log=self.log, stoppingcriterion=reason, outer_iterations=it,
                            inner_iterations=self.inner_total, tcg_iterations=self.tcg_total,
                            matvecs=getattr(P, "matvecs", 0), passes=self.passes,
                            trace=self.trace)


def ripm_operator_aw(P, x, z, s, v):
    """RIPM's condensed Newton operator OperatorAw (src/solver/RIPM.py:485-487) with
    do_euclidean_lincomb=False (RIPM.py:149 default; :399-409): hessLagrangian(x, y, z, dx) =
    rhess f[dx] + sum_i z_i rhess g_i[dx] (:123-132, no equality constraints) plus
    Gx(x, Gxaj(x, dx) * (z / s)) with Gx(x, c) = sum_i c_i rgrad g_i(x) (:12-17) and
    Gxaj(x, dx)_i = <rgrad g_i(x), dx> (:19-24).  RIPM's constraints are the problem's g_i <= 0
    (NonnegPCA: g_i = -x_i) with a separate slack s.  P = NonnegPCAStructured (per-constraint)."""
    vec = P.riemannian_hessian(x, v)
    for i in range(len(z)):
        vec = vec + z[i] * P.ineq_rhess[i](x, v)
    gxaj = np.array([P.manifold.inner_product(x, P.ineq_rgrad[i](x), v) for i in range(len(z))])
    c = gxaj * (z / s)
    theta = P.manifold.zero_vector(x)
    for i in range(len(z)):
        theta = theta + c[i] * P.ineq_rgrad[i](x)
    return vec + theta


def ripm_operator_aw_vectorized(Z, x, z, s, v):
    """Closed form of ripm_operator_aw for NonnegPCA (the HIP kernel's formula):
    Aw(v) = P_x(-S v) + (x^T S x + z^T x)(x^T x) v + P_x((z / s) (v - x (x^T v)))."""
    S = Z + Z.T
    Sx, Sv = S @ x, S @ v
    xx, xSx, zx = x @ x, x @ Sx, z @ x
    coef = (xSx + zx) * xx
    xu, xv = x @ Sv, x @ v
    q = (v - x * xv) * (z / s)
    xq = x @ q
    return ((-Sv + xu * x) + coef * v) + (q - xq * x)


def solve(Z, x0, y0, option=None, structured=False, clock=time.time) -> OracleResult:
    o = option or {}
    P = (NonnegPCAStructured(Z, lincomb=o.get('do_euclidean_lincomb', False),
                             embedded=o.get('is_euclidean_embedded', False))
         if structured else NonnegPCAVectorized(Z))
    return RIPTRMOracle(option, clock=clock).run(P, x0, y0)


def mu_schedule(option: Dict[str, Any], count: int) -> List[float]:
    """Barrier parameters mu_0..mu_{count-1} exactly as RIPTRM.py:852,890-893 produce them."""
    o = default_option()
    o.update(option or {})
    mu = o['initial_barrier_parameter']
    out = []
    for _ in range(count):
        out.append(mu)
        if o['do_simple_barrier_parameter_update']:
            mu = max(o['min_barrier_parameter'],
                     o['barrier_parameter_update_c'] * (mu ** (1 + o['barrier_parameter_update_r'])))
        else:
            mu = max(o['min_barrier_parameter'],
                     min(o['barrier_parameter_update_b'] * mu,
                         o['barrier_parameter_update_c'] * (mu ** (1 + o['barrier_parameter_update_r']))))
    return out
