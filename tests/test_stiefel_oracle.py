"""CPU checks of the Stiefel restatement (oracle/stiefel_oracle.py, pymanopt 2.x formulas; the
reference has no Stiefel problem, so parity is unpinned and these identities are the pin)."""
import numpy as np
import pytest

from oracle.stiefel_oracle import Stiefel, multisym


@pytest.mark.parametrize("n,p", [(5, 1), (12, 4), (200, 50)])
def test_stiefel_identities(n, p):
    M = Stiefel(n, p)
    rs = np.random.RandomState(n + p)
    X = M.random_point(rs)
    assert np.allclose(X.T @ X, np.eye(p), atol=1e-13)
    U = M.projection(X, rs.randn(n, p))
    assert np.allclose(multisym(X.T @ U), 0, atol=1e-13)                   # tangent
    assert np.allclose(M.projection(X, U), U, atol=1e-13)                   # idempotent
    W = rs.randn(n, p)
    assert abs(M.inner_product(X, M.projection(X, W), U) - M.inner_product(X, W, U)) < 1e-10  # self-adjoint
    Y = M.retraction(X, 0.1 * U)
    assert np.allclose(Y.T @ Y, np.eye(p), atol=1e-13)
    assert np.all(np.diag(Y.T @ (X + 0.1 * U)) > 0)   # R = Y^T (X + U) has a positive diagonal (qf)
    # retraction is first-order: R_X(tU) = X + tU + O(t^2)
    t = 1e-6
    assert np.linalg.norm(M.retraction(X, t * U) - X - t * U) < 1e-9
    assert M.dim == n * p - p * (p + 1) // 2 and np.isclose(M.typical_dist, np.sqrt(p))


def test_stiefel_p1_is_the_sphere():
    """Stiefel(n, 1) reduces to the Sphere formulas the NonnegPCA path uses."""
    from oracle.riptrm_oracle import Sphere
    n = 9
    rs = np.random.RandomState(0)
    St, Sp = Stiefel(n, 1), Sphere(n)
    x = Sp.retraction(np.abs(rs.rand(n)), np.zeros(n))
    u = Sp.projection(x, rs.randn(n))
    g, h = rs.randn(n), rs.randn(n)
    X, U = x[:, None], u[:, None]
    assert np.allclose(St.projection(X, rs.randn(n, 1) * 0 + h[:, None])[:, 0], Sp.projection(x, h), atol=1e-14)
    assert np.allclose(St.retraction(X, U)[:, 0], Sp.retraction(x, u), atol=1e-14)
    assert np.allclose(St.euclidean_to_riemannian_hessian(X, g[:, None], h[:, None], U)[:, 0],
                       Sp.euclidean_to_riemannian_hessian(x, g, h, u), atol=1e-13)


def test_rhess_is_self_adjoint_for_a_quadratic():
    """f(X) = -tr(X^T S X)/2: the Riemannian Hessian from e2rh is self-adjoint on T_X St."""
    n, p = 30, 5
    M = Stiefel(n, p)
    rs = np.random.RandomState(3)
    S = rs.randn(n, n)
    S = S + S.T
    X = M.random_point(rs)
    G = -S @ X
    H = lambda V: -S @ V
    U, V = M.random_tangent_vector(X, rs), M.random_tangent_vector(X, rs)
    a = M.inner_product(X, M.euclidean_to_riemannian_hessian(X, G, H(U), U), V)
    b = M.inner_product(X, U, M.euclidean_to_riemannian_hessian(X, G, H(V), V))
    assert abs(a - b) < 1e-11 * max(1, abs(a))
