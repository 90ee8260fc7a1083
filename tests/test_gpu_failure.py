"""Per-instance non-finite guard (include/riptrm.h RIPTRM_ERR_NONFINITE; the device's counterpart of
the reference's do_exit_on_error break, RIPTRM.py:961-966): a NaN / Inf in one instance stops that
instance with an error code and hands back the iterate its outer step started from, while the
other instances of the batch run on exactly as they would alone.  Each case runs through the
persistent path (k_persist) and the lock-step kernels."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from oracle import nonnegpca_gen as G

N, K = 200, 5


def _opt(**kw):
    from problems import manviofun
    o = {"TRS_solver": "tCG", "second_order_stationarity": False, "manviofun": manviofun,
         "tolresid": 0.0, "maxtime": 1e9, "maxiter": K}
    o.update(kw)
    return o


def _insts(B=3, seed=1300):
    return [G.generate_instance(N, seed + b) for b in range(B)]


def _solve(insts, persistent, X0=None, Y0=None):
    import engine
    B = len(insts)
    eng = engine.NonnegPCABatch(N, B, log_capacity=1024, persistent=persistent)
    eng.load_Z(np.stack([z for z, _, _ in insts]))
    X0 = np.stack([x for _, x, _ in insts]) if X0 is None else X0
    Y0 = np.stack([y for _, _, y in insts]) if Y0 is None else Y0
    return eng, eng.solve(X0, Y0, _opt())


def _healthy_match(res, ref, pairs):
    """instances of res (index a) equal those of ref (index b) bitwise"""
    for a, b in pairs:
        assert torch.equal(res.x[a], ref.x[b]) and torch.equal(res.y[a], ref.y[b])
        assert res.stat(a, "ERROR") == 0
        for f in ("OUTER_ITERS", "INNER_ITERS", "TCG_ITERS", "PASSES"):
            assert res.stat(a, f) == ref.stat(b, f), (a, f)
        np.testing.assert_array_equal(np.array(res.log(a)["residual"], float), np.array(ref.log(b)["residual"], float))


@pytest.mark.parametrize("persistent", [1, 0])
def test_nan_in_multiplier_stops_only_that_instance(persistent):
    """y0 with a NaN: the row-0 KKT residual is NaN, the instance stops at the loop head (outer 0)."""
    import engine
    insts = _insts()
    Y0 = np.stack([y for _, _, y in insts])
    Y0[1, 5] = np.nan
    eng, res = _solve(insts, persistent, Y0=Y0)
    assert res.stat(1, "ERROR") == engine.C["RIPTRM_ERR_NONFINITE"]
    assert res.stat(1, "OUTER_ITERS") == 0
    assert res.error(1) is not None and res.stopping_criterion(1) is None
    np.testing.assert_array_equal(res.x[1].cpu().numpy(), insts[1][1])
    assert len(res.log(1)["residual"]) == 1 and np.isnan(res.log(1)["residual"][0])
    _, ref = _solve([insts[0], insts[2]], persistent)
    _healthy_match(res, ref, [(0, 0), (2, 1)])


@pytest.mark.parametrize("persistent", [1, 0])
def test_zero_coordinate_stops_at_tcg_start(persistent):
    """x0 with an exact zero: the barrier gradient mu/x is infinite, ||cxCur|| is not finite at the
    first tCG start (outer iteration 1); the instance returns the outer step's start point."""
    import engine
    insts = _insts(seed=1310)
    X0 = np.stack([x for _, x, _ in insts])
    X0[2, 7] = 0.0
    X0[2] /= np.linalg.norm(X0[2])
    eng, res = _solve(insts, persistent, X0=X0)
    assert res.stat(2, "ERROR") == engine.C["RIPTRM_ERR_NONFINITE"]
    assert res.stat(2, "OUTER_ITERS") == 1
    np.testing.assert_array_equal(res.x[2].cpu().numpy(), X0[2])
    np.testing.assert_array_equal(res.y[2].cpu().numpy(), insts[2][2])
    _, ref = _solve(insts[:2], persistent)
    _healthy_match(res, ref, [(0, 0), (1, 1)])


@pytest.mark.parametrize("persistent", [1, 0])
def test_inf_multiplier_stops_tcg(persistent):
    """riptrm_tcg with y containing +Inf: cxCur does not involve y, so tCG starts, and the first
    <delta, H delta> is not finite -> stop code NONFINITE for that instance only."""
    import engine
    Z, _, _ = G.generate_instance(N, 1320)
    B = 3
    rs = np.random.RandomState(9)
    xs = np.abs(rs.rand(B, N))
    xs /= np.linalg.norm(xs, axis=1, keepdims=True)
    ys = rs.rand(B, N) + 0.1
    bad = ys.copy()
    bad[1, 3] = np.inf
    out = []
    for y in (bad, ys):
        eng = engine.NonnegPCABatch(N, B, persistent=persistent)
        eng.load_Z(np.broadcast_to(Z, (B, N, N)))
        out.append(eng.tcg(xs, y, 1e-2, np.pi / 8))
    (e1, h1, j1, s1), (e0, h0, j0, s0) = out
    assert s1[1] == "NONFINITE" and s0[1] != "NONFINITE"
    for b in (0, 2):
        assert torch.equal(e1[b], e0[b]) and j1[b] == j0[b] and s1[b] == s0[b]
