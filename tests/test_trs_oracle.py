"""CPU tests of the Exact_RepMat restatement (oracle/trs_oracle.py).

TRSgep (RIPTRM.py:218-299) is restated twice: `trs_gep` with the reference's 2n x 2n pencil and
SciPy's CG, and `trs_eigh`, the symmetric-eigendecomposition + secular-equation form the HIP
kernel computes.  They must agree on random easy, interior and hard-case subproblems; the tangent
basis must be orthonormal in the SI product metric, and the represented matrix must reproduce the
operator (utils.py:565-573).  The reference's own tangent basis is random (utils.py:388-397), so
no golden vector of a TRS direction exists: agreement is checked by optimality, not by fixture."""
import os

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import si_oracle as SI
from oracle import trs_oracle as T

DS = os.path.join(GOLDEN, "si_1")


def _obj(A, a, x):
    return 0.5 * x @ A @ x + a @ x


@pytest.mark.parametrize("seed", range(6))
def test_eigh_form_matches_pencil_form(seed):
    rs = np.random.RandomState(seed)
    for t in range(25):
        n = rs.randint(2, 41)
        M = rs.randn(n, n)
        A = M @ M.T + 0.1 * np.eye(n) if t % 3 == 0 else M + M.T
        a = rs.randn(n)
        Del = 10 ** rs.uniform(-2, 1)
        x1, l1, k1 = T.trs_gep(A, a, Del, 1e-8)
        x2, l2, k2 = T.trs_eigh(A, a, Del, 1e-8)
        assert k1 == k2
        assert np.linalg.norm(x1 - x2) <= 1e-8 * np.linalg.norm(x1)
        assert abs(l1 - l2) <= 1e-8 * max(1.0, abs(l1))
        # KKT of the TRS: (A + lam I) x = -a, lam >= 0 on the boundary, A + lam I PSD
        if k2 == "boundary":
            assert abs(np.linalg.norm(x2) - Del) <= 1e-12 * Del
            assert np.linalg.norm(A @ x2 + l2 * x2 + a) <= 1e-8 * np.linalg.norm(a)
            assert np.linalg.eigvalsh(A + l2 * np.eye(n))[0] >= -1e-9 * max(1.0, abs(l2))


def test_hard_case():
    rs = np.random.RandomState(7)
    for _ in range(5):
        n = 9
        Q, _ = np.linalg.qr(rs.randn(n, n))
        lam = np.sort(rs.randn(n))
        lam[0] = -3.0
        A = Q @ np.diag(lam) @ Q.T
        g = rs.randn(n)
        g[0] = 0.0
        a = Q @ g
        x1, l1, k1 = T.trs_gep(A, a, 5.0, 1e-8)
        x2, l2, k2 = T.trs_eigh(A, a, 5.0, 1e-8)
        assert k1 == k2 == "hardcase_1"
        assert np.isclose(l1, 3.0) and np.isclose(l2, 3.0)
        # the hard-case sign of the q_min component is arbitrary in both: compare objective values
        assert np.isclose(_obj(A, a, x1), _obj(A, a, x2), rtol=1e-12)
        assert np.isclose(np.linalg.norm(x2), 5.0)


def test_scipy_cg_restatement_matches_scipy():
    import scipy.sparse.linalg
    rs = np.random.RandomState(3)
    for n in (3, 17, 40):
        M = rs.randn(n, n)
        A = M @ M.T + np.eye(n)
        b = rs.randn(n)
        ref, _ = scipy.sparse.linalg.cg(A, b)
        assert np.allclose(T.scipy_cg(A, b), ref, rtol=1e-12, atol=1e-14)


def test_si_tangent_basis_orthonormal_and_represents_hw():
    data = SI.SIData.load(DS)
    P = SI.SIVectorized(data)
    M = P.manifold
    x, y = SI.load_start(DS, "c")
    B = T.si_tangent_basis(x)
    assert len(B) == M.dim == 40
    G = np.array([[M.inner_product(x, bi, bj) for bj in B] for bi in B])
    assert np.allclose(G, np.eye(40), atol=1e-12)
    for b in B:
        assert np.allclose(M.projection(x, b), b, atol=1e-12)
    _, _, Hw, c = P.begin_inner(x, y, 0.01)
    H = T.selfadj_operator2matrix(M, x, Hw, B)
    assert np.allclose(H, H.T)
    coef = np.random.RandomState(5).randn(40)
    v = sum(ci * bi for ci, bi in zip(coef, B))
    Hv = np.array([M.inner_product(x, Hw(v), b) for b in B])
    assert np.allclose(Hv, H @ coef, rtol=1e-9, atol=1e-9 * np.abs(Hv).max())


def test_si_exact_repmat_oracle_short_run():
    data = SI.SIData.load(DS)
    x0, y0 = SI.load_start(DS, "a")
    r = SI.solve(data, x0, y0, dict(maxiter=1, tolresid=0, maxtime=1e9, TRS_solver="Exact_RepMat",
                                     second_order_stationarity=True))
    kinds = [k for k in r.log["dxtype"] if k is not None]
    assert kinds and all(k in ("boundary", "interior") or k.startswith("hardcase") for k in kinds)
    mins = [v for v in r.log["mineigvalHw"] if v is not None]
    assert mins and all(np.isfinite(mins))


def test_sphere_basis_and_direction_are_basis_independent(fixture_n50):
    """NonnegPCA: the Householder frame (device) and the reference's random Gram-Schmidt frame
    (utils.py:388-397) give the same Exact_RepMat direction and the same smallest eigenvalue."""
    from oracle import riptrm_oracle as O
    Z, x0, y0 = fixture_n50
    P = O.NonnegPCAVectorized(Z)
    M = P.manifold
    _, _, Hw, c = P.begin_inner(x0 / np.linalg.norm(x0), y0, 0.1)
    x = x0 / np.linalg.norm(x0)
    Bh = O.sphere_tangent_basis(x)
    Br = O.sphere_tangent_basis(x, np.random.RandomState(0))
    for B in (Bh, Br):
        G = np.array([[bi @ bj for bj in B] for bi in B])
        assert np.allclose(G, np.eye(len(B)), atol=1e-12)
        assert max(abs(b @ x) for b in B) < 1e-12
    d1, _, k1, H1 = T.exact_repmat_direction(M, x, Hw, c, 0.3, Bh, 1e-8)
    d2, _, k2, H2 = T.exact_repmat_direction(M, x, Hw, c, 0.3, Br, 1e-8)
    assert k1 == k2
    assert np.linalg.norm(d1 - d2) <= 1e-8 * np.linalg.norm(d1)
    assert abs(np.linalg.eigvalsh(H1)[0] - np.linalg.eigvalsh(H2)[0]) <= 1e-10 * np.abs(H1).max()


def test_nonnegpca_exact_repmat_oracle_short_run(fixture_n50):
    from oracle import riptrm_oracle as O
    Z, x0, y0 = fixture_n50
    r = O.solve(Z, x0, y0, dict(maxiter=3, tolresid=0, maxtime=1e9, TRS_solver="Exact_RepMat",
                                second_order_stationarity=True, manviofun=O.sphere_manvio))
    kinds = [k for k in r.log["dxtype"] if k is not None]
    assert kinds and all(k in ("boundary", "interior") or k.startswith("hardcase") for k in kinds)
    assert r.log["residual"][-1] < r.log["residual"][0]
