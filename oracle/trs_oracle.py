"""Exact_RepMat trust-region subproblem path — TEST INFRASTRUCTURE ONLY.

Restates, for the checker of the HIP implementation:
  * TRSgep (src/solver/RIPTRM.py:218-299): min x^T A x / 2 + a^T x s.t. x^T B x <= Delta^2 through
    the rightmost eigenpair of the 2n x 2n pencil (MM0, -MM1), with the interior candidate from
    SciPy's CG (RIPTRM.py:245-251) and the hard-case refinement (:266-291); B = I at the call
    site (RIPTRM.py:441).
  * selfadj_operator2matrix (src/solver/utils.py:565-573): the operator in a tangent basis.
  * compute_direction's Exact_RepMat branch (RIPTRM.py:433-444) and the second-order
    stationarity test (RIPTRM.py:599-617).
The reference draws its tangent basis at random (utils.py:388-397, unseeded); the TRS solution is
basis-independent, so the checker uses a deterministic orthonormal basis (`si_tangent_basis`).
"""
from __future__ import annotations

import numpy as np
import scipy.linalg
import scipy.sparse.linalg


def selfadj_operator2matrix(M, x, F, basis):
    """utils.py:565-573: A[i, j] = <b_i, F(b_j)> for i <= j, mirrored."""
    n = len(basis)
    A = np.zeros((n, n))
    for j in range(n):
        Fb = F(basis[j])
        for i in range(j + 1):
            A[i, j] = M.inner_product(x, Fb, basis[i])
    return A + np.triu(A, 1).T


def trs_gep(A, a, Del, tolhardcase=1e-4):
    """RIPTRM.py:218-299 with B = I.  Returns (x, lam1, type)."""
    n = A.shape[0]
    B = np.eye(n)
    MM0 = np.block([[-B, A], [A, -np.outer(a, a) / (Del ** 2)]])
    MM1 = np.block([[np.zeros((n, n)), B], [B, np.zeros((n, n))]])
    p1, _ = scipy.sparse.linalg.cg(A, -a)                     # interior candidate (:245)
    if np.linalg.norm(A @ p1 + a) / np.linalg.norm(a) < 1e-5:
        if p1 @ B @ p1 >= Del ** 2:
            p1 = np.full_like(p1, np.nan)
    else:
        p1 = np.full_like(p1, np.nan)
    lams, vecs = scipy.linalg.eig(a=MM0, b=-MM1)               # rightmost eigenpair (:254-259)
    k = np.argmax(np.real(lams))
    lam1 = np.real(lams[k])
    V = np.real(vecs[:, k])
    x = V[:n]
    normx = np.sqrt(x @ (B @ x))
    x = x / normx * Del
    if x @ a > 0:
        x = -x
    kind = "boundary"
    if normx < tolhardcase:                                    # hard case (:266-291)
        x1 = V[n:]
        Alam1B = A + lam1 * B
        BP = B @ x1
        H = Alam1B + lam1 * np.outer(BP, BP)
        x2 = scipy.linalg.solve(H, -a, assume_a='sym')
        kind = "hardcase_1"
        if np.linalg.norm(Alam1B @ x2 + a) / np.linalg.norm(a) > tolhardcase:
            _, v = scipy.linalg.eigh(A, B)
            for ii in [3, 6, 9]:
                P = v[:, :ii]
                BP = B @ P
                H = Alam1B + lam1 * BP @ BP.T
                x2 = scipy.linalg.solve(H, -a, assume_a='sym')
                kind = f"hardcase_{ii}"
                if np.linalg.norm(Alam1B @ x2 + a) / np.linalg.norm(a) < tolhardcase:
                    break
        aa = x1 @ (B @ x1)
        bb = 2 * x2 @ (B @ x1)
        cc = x2 @ (B @ x2) - Del ** 2
        alp = (-bb + np.sqrt(bb ** 2 - 4 * aa * cc)) / (2 * aa)
        x = x2 + alp * x1
    if not np.isnan(p1).any():                                 # interior vs boundary (:294-298)
        if 0.5 * (p1 @ A @ p1) + a @ p1 <= 0.5 * (x @ A @ x) + a @ x:
            x = p1
            lam1 = 0
            kind = "interior"
    return x, lam1, kind


def si_tangent_basis(x):
    """Orthonormal basis of T_x(Skew(d) x SPD(d) x SPD(d)) in the product metric, deterministic:
    skew pairs (E_ij - E_ji)/sqrt2 (i < j), then for R and Q the images L B_k L^T of the Frobenius-
    orthonormal symmetric basis B_k = E_ii, (E_ij + E_ji)/sqrt2 (i < j) under the Cholesky factor
    L of the point (<L B L^T, L C L^T>_X = tr(B C) for the affine-invariant metric)."""
    d = x.shape[1]
    out = []
    for i in range(d):
        for j in range(i + 1, d):
            b = np.zeros((3, d, d))
            b[0, i, j] = 1 / np.sqrt(2)
            b[0, j, i] = -1 / np.sqrt(2)
            out.append(b)
    for comp in (1, 2):
        L = np.linalg.cholesky(x[comp])
        for i in range(d):
            for j in range(i, d):
                Bk = np.zeros((d, d))
                if i == j:
                    Bk[i, i] = 1.0
                else:
                    Bk[i, j] = Bk[j, i] = 1 / np.sqrt(2)
                b = np.zeros((3, d, d))
                b[comp] = L @ Bk @ L.T
                out.append(b)
    return out


def exact_repmat_direction(M, x, Hw, c, Delta, basis, tolhardcase):
    """compute_direction, Exact_RepMat branch (RIPTRM.py:433-444): returns (dx, lam1, type, H)."""
    H = selfadj_operator2matrix(M, x, Hw, basis)
    cv = np.array([M.inner_product(x, c, b) for b in basis])
    coeff, lam1, kind = trs_gep(H, cv, Delta, tolhardcase)
    dx = M.zero_vector(x)
    for i in range(len(basis)):
        dx = dx + coeff[i] * basis[i]
    return dx, lam1, kind, H


def scipy_cg(A, b, rtol=1e-5):
    """The CG iteration of scipy.sparse.linalg.cg (SciPy 1.15, x0 = 0, no preconditioner,
    maxiter = 10 n) as TRSgep calls it (RIPTRM.py:245), restated loop for loop so the device
    kernel (csrc/riptrm_si.hip, Eng::trs_cg) can mirror it."""
    n = len(b)
    x = np.zeros(n)
    bnrm2 = np.linalg.norm(b)
    if bnrm2 == 0:
        return b.copy()
    atol = rtol * bnrm2
    r = b.copy()
    p = None
    rho_prev = None
    for it in range(10 * n):
        if np.linalg.norm(r) < atol:
            return x
        rho = r @ r
        if it > 0:
            p = p * (rho / rho_prev) + r
        else:
            p = r.copy()
        q = A @ p
        alpha = rho / (p @ q)
        x = x + alpha * p
        r = r - alpha * q
        rho_prev = rho
    return x


def trs_eigh(A, a, Del, tolhardcase=1e-8):
    """The device formulation of TRSgep (B = I): the same three candidates, computed from the
    symmetric eigendecomposition A = Q diag(lam) Q^T instead of the 2n x 2n pencil.  The pencil's
    rightmost eigenvalue is the rightmost root lam1 of ||(A + lam I)^-1 a|| = Del on
    (-lam_min, inf) (Adachi et al. 2017), so in the easy case the boundary candidate is
    -(A + lam1 I)^-1 a; the root is found by safeguarded Newton on 1/||x(lam)|| - 1/Del.  Hard
    case (a orthogonal to the lam_min eigenspace): lam1 = -lam_min, x = x2 + alp q_min with
    alp = +sqrt(Del^2 - ||x2||^2) (RIPTRM.py:286-291 with x1 = q_min, x1 ⟂ x2).
    Returns (x, lam1, type)."""
    n = A.shape[0]
    p1 = scipy_cg(A, -a)
    na = np.linalg.norm(a)
    ok = na > 0 and np.linalg.norm(A @ p1 + a) / na < 1e-5 and p1 @ p1 < Del ** 2
    lam, Q = np.linalg.eigh(A)
    g = Q.T @ a
    lmin = lam[0]
    hard_set = np.abs(lam - lmin) <= 1e-12 * max(1.0, np.abs(lam).max())
    ghard = np.sqrt(np.sum(g[hard_set] ** 2))
    lo = -lmin
    gn = np.linalg.norm(g)
    if ghard <= tolhardcase * gn:
        d = lam[~hard_set] - lmin
        x2c = np.zeros(n)
        x2c[~hard_set] = -g[~hard_set] / d
        if x2c @ x2c < Del ** 2:
            kind = "hardcase_1"
            alp = np.sqrt(Del ** 2 - x2c @ x2c)
            x = Q @ x2c + alp * Q[:, 0]
            lam1 = lo
            return _pick_interior(A, a, p1, ok, x, lam1, kind)
    hi = lo + gn / Del
    l1 = hi
    for _ in range(100):
        den = lam + l1
        xn = np.sqrt(np.sum((g / den) ** 2))
        f = 1.0 / xn - 1.0 / Del
        fp = np.sum(g ** 2 / den ** 3) / xn ** 3
        step = f / fp
        nl = l1 - step
        if nl <= lo:
            nl = 0.5 * (lo + l1)
        if abs(nl - l1) <= 1e-15 * max(1.0, abs(l1)):
            l1 = nl
            break
        l1 = nl
    x = Q @ (-g / (lam + l1))
    x = x / np.linalg.norm(x) * Del
    return _pick_interior(A, a, p1, ok, x, l1, "boundary")


def _pick_interior(A, a, p1, ok, x, lam1, kind):
    if ok and 0.5 * (p1 @ A @ p1) + a @ p1 <= 0.5 * (x @ A @ x) + a @ x:   # RIPTRM.py:294-298
        return p1, 0.0, "interior"
    return x, lam1, kind
