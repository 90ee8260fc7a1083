"""CPU tests of the oracle (the parity checker) against the reference's known answers and
internal consistency.  No GPU needed."""
import numpy as np
import pytest

from oracle import nonnegpca_gen as G
from oracle import riptrm_oracle as O

OPT = dict(tolresid=0.0, maxtime=1e9, manviofun=O.sphere_manvio)


def _eval0(P, x0, y0):
    orc = O.RIPTRMOracle(dict(OPT))
    return orc.evaluation(P, x0, x0, y0)


@pytest.mark.parametrize("structured", [False, True])
def test_initial_residual_known_answer(fixture_n50, structured):
    """src/NonnegPCA/analyzer.ipynb (cell 5 output): every solver's row 0 on dataset/NonnegPCA/1,
    point a, has KKT residual 4.986888e+00."""
    Z, x0, y0 = fixture_n50
    P = O.NonnegPCAStructured(Z) if structured else O.NonnegPCAVectorized(Z)
    ev = _eval0(P, x0, y0)
    assert f"{ev['residual']:.6e}" == "4.986888e+00"


def test_fixture_run_reaches_published_residual(fixture_n50):
    """analyzer.ipynb cell 5 plot: RIPTRM (tCG) reaches ~1e-14 KKT residual and stays flat."""
    Z, x0, y0 = fixture_n50
    r = O.solve(Z, x0, y0, dict(OPT, maxiter=45))
    res = np.array(r.log["residual"], dtype=float)
    conv = [i for i, s in enumerate(r.log["inner_status"]) if s in (None, "converged")]
    rc = res[conv]
    assert rc[-1] < 2e-14
    # the converged-row residual decreases over the first ~35 outer iterations
    assert np.all(np.diff(np.log10(rc[:36])) < 0)
    assert r.stoppingcriterion.startswith("Max iteration count reached; maxiter=45")


def test_structured_matches_vectorized_fixture(fixture_n50):
    Z, x0, y0 = fixture_n50
    a = O.solve(Z, x0, y0, dict(OPT, maxiter=8), structured=True)
    b = O.solve(Z, x0, y0, dict(OPT, maxiter=8), structured=False)
    assert a.log["inner_status"] == b.log["inner_status"]
    assert a.log["dxtype"] == b.log["dxtype"]
    # trajectory-level: summation-order differences are amplified by tCG, ~1e-8 relative here
    np.testing.assert_allclose(np.array(a.log["residual"], float), np.array(b.log["residual"], float),
                               rtol=1e-6, atol=1e-14)
    np.testing.assert_allclose(a.x, b.x, atol=1e-7)
    np.testing.assert_allclose(a.y, b.y, rtol=1e-5, atol=1e-8)


def test_barrier_hessian_closed_form_matches_structured():
    rs = np.random.RandomState(3)
    n = 23
    Z = rs.randn(n, n)
    x = np.abs(rs.rand(n)); x /= np.linalg.norm(x)
    y = rs.rand(n) + 0.1
    mu = 0.03
    Ps, Pv = O.NonnegPCAStructured(Z), O.NonnegPCAVectorized(Z)
    _, s1, H1, c1 = Ps.begin_inner(x, y, mu)
    _, s2, H2, c2 = Pv.begin_inner(x, y, mu)
    np.testing.assert_allclose(c1, c2, rtol=1e-12, atol=1e-13)
    for _ in range(3):
        v = Ps.manifold.projection(x, rs.randn(n))
        np.testing.assert_allclose(H1(v), H2(v), rtol=1e-11, atol=1e-12)
    np.testing.assert_allclose(Ps.gradlag(x, y), Pv.gradlag(x, y), rtol=1e-12, atol=1e-13)


def test_gradient_matches_torch_autograd():
    torch = pytest.importorskip("torch")
    rs = np.random.RandomState(5)
    n = 17
    Z = rs.randn(n, n)
    x = rs.randn(n)
    xt = torch.tensor(x, requires_grad=True)
    f = -(xt @ torch.tensor(Z) @ xt)
    (g,) = torch.autograd.grad(f, xt, create_graph=True)
    v = rs.randn(n)
    (hv,) = torch.autograd.grad(g @ torch.tensor(v), xt)
    P = O.NonnegPCAVectorized(Z)
    np.testing.assert_allclose(-P.S @ x, g.detach().numpy(), rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(-P.S @ v, hv.numpy(), rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(O.NonnegPCAStructured(Z).euclidean_gradient(x), g.detach().numpy(), atol=1e-12)


def test_riemannian_hessian_finite_difference():
    """Hess f[v] = P(ehess[v]) + W(x, v, normal egrad) (pymanopt Sphere) vs a central difference
    of the Riemannian gradient along the retraction curve (second-order accurate on the sphere)."""
    rs = np.random.RandomState(11)
    n = 12
    Z = rs.randn(n, n)
    P = O.NonnegPCAStructured(Z)
    M = P.manifold
    x = rs.randn(n); x /= np.linalg.norm(x)
    v = M.projection(x, rs.randn(n))
    h = 1e-5
    gp = P.riemannian_gradient(M.retraction(x, h * v))
    gm = P.riemannian_gradient(M.retraction(x, -h * v))
    fd = M.projection(x, (gp - gm) / (2 * h))
    np.testing.assert_allclose(P.riemannian_hessian(x, v), fd, rtol=1e-6, atol=1e-6)


def test_tcg_invariants():
    rs = np.random.RandomState(7)
    n = 40
    Z, x0, y0 = G.generate_instance(n, 99)
    P = O.NonnegPCAVectorized(Z)
    M = P.manifold
    seen = set()
    for Delta in (1e-3, 0.05, 0.4, 3.0):
        for mu in (0.1, 1e-3):
            _, s, Hw, c = P.begin_inner(x0, y0, mu)
            eta, Heta, j, stop = O.truncated_conjugate_gradient(M, Hw, x0, c, Delta, 1, 0.1, 1, M.dim)
            seen.add(stop)
            assert np.linalg.norm(eta) <= Delta * (1 + 1e-10)
            model = M.inner_product(x0, eta, c) + 0.5 * M.inner_product(x0, eta, Hw(eta))
            assert model <= 1e-14
            if stop in ("EXCEEDED_TR", "NEGATIVE_CURVATURE"):
                assert abs(np.linalg.norm(eta) - Delta) <= 1e-9 * Delta
            assert abs(x0 @ eta) < 1e-10  # tangent
            assert 0 <= j < M.dim
    assert "EXCEEDED_TR" in seen


def test_mu_schedule_matches_engine_table():
    import engine
    o = dict(engine.REFERENCE_DEFAULTS)
    tab = engine.mu_schedule(o, 100)
    ref = O.mu_schedule({}, len(tab))
    assert tab == ref                                  # bit-exact Python floats
    assert tab[0] == 0.1 and tab[-1] == 1e-15
    k20 = tab[20]
    assert 1.3e-8 < k20 < 1.5e-8                       # mu_20 ~ 1.42e-8
    assert 36 <= len(tab) <= 41                        # floor 1e-15 after ~38 updates


def test_generator_recipe_properties():
    Z1, x1, y1 = G.generate_instance(60, 5)
    Z2, x2, y2 = G.generate_instance(60, 5)
    np.testing.assert_array_equal(Z1, Z2)
    assert np.all(x1 >= 0) and abs(np.linalg.norm(x1) - 1) < 1e-14
    assert np.all(y1 == 1)
    Z3, _, _ = G.generate_instance(60, 6)
    assert not np.array_equal(Z1, Z3)


def test_oracle_edge_paths():
    """inner_maxiter reset path (RIPTRM.py:835-842), save_inner_iteration=False rows, tiny n."""
    Z, x0, y0 = G.generate_instance(6, 1)
    r = O.solve(Z, x0, y0, dict(OPT, maxiter=3, inner_maxiter=1))
    assert r.outer_iterations == 3
    r2 = O.solve(Z, x0, y0, dict(OPT, maxiter=4, save_inner_iteration=False))
    assert r2.log["iteration"] == [0, 1, 2, 3, 4]
    assert "dxtype" not in r2.log
    Z, x0, y0 = G.generate_instance(2, 1)
    r3 = O.solve(Z, x0, y0, dict(OPT, maxiter=5))
    assert r3.outer_iterations == 5


@pytest.mark.parametrize("n,seed,K", [(37, 100, 10), (37, 101, 10), (37, 104, 10), (200, 101, 12)])
def test_comparator_calibration(n, seed, K):
    """The GPU parity bar (tests/parity.py) is met by the two CPU oracles against each other:
    it is the size of fp64 summation-order noise on these trajectories, not looser."""
    from parity import compare_logs
    Z, x0, y0 = G.generate_instance(n, seed)
    a = O.solve(Z, x0, y0, dict(OPT, maxiter=K), structured=True)
    b = O.solve(Z, x0, y0, dict(OPT, maxiter=K))
    compare_logs(a.log, b.log)


@pytest.mark.parametrize("n,seed,K", [(37, 125, 10), (60, 115, 10)])
def test_outer_comparator_on_branch_flips(n, seed, K):
    """On instances where the two CPU oracles' inner branches differ, the outer-level comparator
    (used for the same situation on the GPU) holds."""
    from parity import BranchFlip, compare_logs, compare_outer
    Z, x0, y0 = G.generate_instance(n, seed)
    a = O.solve(Z, x0, y0, dict(OPT, maxiter=K), structured=True)
    b = O.solve(Z, x0, y0, dict(OPT, maxiter=K))
    with pytest.raises(BranchFlip):
        compare_logs(a.log, b.log)
    compare_outer(a.log, b.log)


def test_ripm_operator_aw_closed_form():
    """RIPM OperatorAw (RIPM.py:485-487): per-constraint wiring == closed form,
    and the operator is self-adjoint on the tangent space."""
    from oracle import nonnegpca_gen as G2
    Z, x0, _ = G2.generate_instance(23, 77)
    rs = np.random.RandomState(1)
    x = x0 / np.linalg.norm(x0)
    z = rs.rand(23) + 0.1
    s = rs.rand(23) + 0.2
    P = O.NonnegPCAStructured(Z)
    u = P.manifold.projection(x, rs.randn(23))
    w = P.manifold.projection(x, rs.randn(23))
    a = O.ripm_operator_aw(P, x, z, s, u)
    b = O.ripm_operator_aw_vectorized(Z, x, z, s, u)
    assert np.linalg.norm(a - b) <= 1e-12 * np.linalg.norm(a)
    l = P.manifold.inner_product(x, O.ripm_operator_aw(P, x, z, s, u), w)
    r = P.manifold.inner_product(x, u, O.ripm_operator_aw(P, x, z, s, w))
    assert abs(l - r) <= 1e-11 * max(1.0, abs(l))


@pytest.mark.parametrize("lincomb,embedded", [(True, False), (False, True), (True, True)])
def test_euclidean_branch_options_agree(lincomb, embedded):
    """do_euclidean_lincomb / is_euclidean_embedded (RIPTRM.py:480-482, :514-517, :543-545,
    :567-568) restated per constraint: on the Sphere they compute the default branches' operators
    (linear conversions; x^T dx = 0 for tangent dx), so the whole trajectory matches the default
    one at the summation-order bar, and the device's closed form (which serves all four option
    combinations) stands for each of them."""
    from parity import compare_logs
    Z, x0, y0 = G.generate_instance(37, 100)
    opt = dict(OPT, maxiter=8, do_euclidean_lincomb=lincomb, is_euclidean_embedded=embedded)
    a = O.solve(Z, x0, y0, opt, structured=True)
    b = O.solve(Z, x0, y0, dict(OPT, maxiter=8), structured=True)
    c = O.solve(Z, x0, y0, dict(OPT, maxiter=8))
    compare_logs(a.log, b.log)
    compare_logs(a.log, c.log)
    P = O.NonnegPCAStructured(Z, lincomb=lincomb, embedded=embedded)
    Q = O.NonnegPCAStructured(Z)
    rs = np.random.RandomState(3)
    x = x0 / np.linalg.norm(x0)
    y = rs.rand(37) + 0.1
    u = Q.manifold.projection(x, rs.randn(37))
    _, _, Hp, cp = P.begin_inner(x, y, 0.01)
    _, _, Hq, cq = Q.begin_inner(x, y, 0.01)
    assert np.linalg.norm(Hp(u) - Hq(u)) <= 1e-12 * np.linalg.norm(Hq(u))
    assert np.linalg.norm(cp - cq) <= 1e-12 * np.linalg.norm(cq)
    assert np.linalg.norm(P.gradlag(x, y) - Q.gradlag(x, y)) <= 1e-12 * np.linalg.norm(Q.gradlag(x, y))


def test_envelope_calibration():
    """parity.compare_logs(envelope=...) as the GPU solve tests use it, with CPU stand-ins for the
    GPU: further order variants (dsymv on other permutations) and the reference-structured oracle
    against the dsymv oracle, the envelope made of parity.order_variants' five runs.  No stand-in
    may fail the bar; envelope excursions (trial values past 10x the envelope but inside the
    calibrated bound) stay within parity.excursion_budget of the comparisons; the tCG exit
    indices meet compare_tcg_iters.  (Measured while choosing the bar: the row-level 3x envelope
    of three variants is exceeded by up to 470x, the column-level one by up to 8.2x; with five
    variants and 10x, 1 comparison of 44 had an excursion, n = 37 seed 108, minyfeasi.)"""
    from parity import (BranchFlip, compare_logs, compare_tcg_iters, envelope, excursion_budget,
                        order_variants)
    cases = [(37, s) for s in range(100, 112)] + [(60, s) for s in (110, 111, 113)]
    compared, exc = 0, []
    for n, seed in cases:
        Z, x0, y0 = G.generate_instance(n, seed)
        opt = dict(OPT, maxiter=10)
        ref = O.RIPTRMOracle(opt).run(O.NonnegPCAVectorized(Z), x0, y0)
        env = envelope(ref, order_variants(Z, x0, y0, opt))
        S = Z + Z.T
        for sd in (3, 4, "structured"):
            if sd == "structured":
                r = O.RIPTRMOracle(opt).run(O.NonnegPCAStructured(Z), x0, y0)
            else:
                p = np.random.RandomState(sd).permutation(n)
                Sp = np.ascontiguousarray(S[p][:, p])
                r = O.RIPTRMOracle(opt).run(O.NonnegPCAVectorized(Sp, S=Sp), x0[p], y0[p])
            e = []
            try:
                compare_logs(r.log, ref.log, envelope=env, excursions=e)
            except BranchFlip:
                continue
            compare_tcg_iters([t["tcg_iters"] for t in r.trace], ref, env)
            compared += 1
            if e:
                exc.append((n, seed, sd, e))
    assert compared >= 30
    assert len(exc) <= excursion_budget(compared), exc


def test_parallel_checker_matches_sequential():
    """parity.check_instances_parallel (the n = 4000 GPU tests' pool of single-threaded oracle
    processes) reaches the same verdict as parity.check_instance: here the 'GPU' log is the
    reference-structured oracle's, one instance that agrees and one whose branches flip (seed 125,
    test_outer_comparator_on_branch_flips)."""
    from parity import check_instance, check_instances_parallel, null_summary
    opt = dict(OPT, maxiter=10)
    items = []
    for n, seed in ((37, 100), (37, 125)):
        Z, x0, y0 = G.generate_instance(n, seed)
        a = O.solve(Z, x0, y0, opt, structured=True)
        items.append(dict(gl=a.log, S=Z + Z.T, x0=x0, y0=y0, gpu_x=a.x, gpu_y=a.y, name=seed, Z=Z))
    msgs = []
    par = check_instances_parallel(items, opt, workers=2, progress=msgs.append)
    assert len(msgs) >= 2
    for it in items:
        seq = check_instance(it["gl"], it["Z"], it["x0"], it["y0"], opt, it["gpu_x"], it["gpu_y"])
        for key in ("div_row", "dx", "dy", "outer_dev"):
            assert seq["gpu"][key] == par[it["name"]]["gpu"][key], key
            assert seq["u_" + key] == par[it["name"]]["u_" + key], key
    assert par[125]["gpu"]["flip"] is not None and par[100]["gpu"]["flip"] is None
    assert null_summary([par[100], par[125]])["ok"]


class _HessianError(O.NonnegPCAVectorized):
    """Negative control for the null test: every S.v carries a fixed relative error of size `rel`
    (elementwise factors 1 +- rel), a systematic defect a kernel could have while still passing an
    operator-level 1e-8 check."""

    def __init__(self, S, rel, seed):
        super().__init__(S, S=S)
        self.w = 1.0 + rel * np.random.RandomState(seed).choice([-1.0, 1.0], size=S.shape[0])

    def Sv(self, v):
        return super().Sv(v) * self.w


def test_null_calibration_accepts_variants_and_rejects_hessian_error():
    """parity.null_row / null_summary, the round-5 bar of the GPU trajectory tests, calibrated on the
    CPU over the regime the bench window lives in (K = 20 outer iterations, mu down to 1.4e-8, where
    every summation-order variant leaves the reference run's branches somewhere: n = 100, 14
    instances, 6 variants each):
    * null: each variant in the GPU's place against the other five (leave_one_out) passes -- the
      bar's false-alarm level is what it claims;
    * power at the sizes the GPU tests use: a run whose Hessian action carries a 1e-9 relative error
      (_HessianError) fails against 4 variants (the SI test) and 5 (the NonnegPCA tests) at 11, 12
      and 14 instances (the pooled GPU tests: 12 SI / configs[1] / multi-start instances, 14 at
      n = 4000, 16 batched), and even at 6 and 8 (it is the strictly earliest-diverging run on nearly
      every instance).  assert_null refuses fewer instances than give a mean-u limit above 0.2
      (parity.NULL_U_MIN_FLOOR).  Measured while choosing the pooling (16 instances): a 1e-10 error
      fails from 8 instances on, a 1e-12 one (rounding level) passes at every size."""
    from parity import NULL_U_MIN_FLOOR, leave_one_out, null_row, null_summary, run_divergence
    opt = dict(OPT, maxiter=20)
    variants, bad = [], []
    for s in range(14):
        Z, x0, y0 = G.generate_instance(100, 7000 + s)
        S = Z + Z.T
        ref = O.RIPTRMOracle(opt).run(O.NonnegPCAVectorized(S, S=S), x0, y0)
        runs = []
        r = O.RIPTRMOracle(opt).run(O.NonnegPCAVectorized(S, S=S, symv=False), x0, y0)
        runs.append(run_divergence(r.log, r.x, r.y, ref.log, ref.x, ref.y))
        for sd in (1, 2, 6, 7, 3):
            p = np.random.RandomState(sd).permutation(100)
            inv = np.argsort(p)
            Sp = np.ascontiguousarray(S[p][:, p])
            r = O.RIPTRMOracle(opt).run(O.NonnegPCAVectorized(Sp, S=Sp), x0[p], y0[p])
            runs.append(run_divergence(r.log, r.x[inv], r.y[inv], ref.log, ref.x, ref.y))
        variants.append(runs)
        r = O.RIPTRMOracle(opt).run(_HessianError(S, 1e-9, 7000 + s), x0, y0)
        bad.append(run_divergence(r.log, r.x, r.y, ref.log, ref.x, ref.y))
    assert all(v["div_row"] < v["rows"] for runs in variants for v in runs)   # the flip regime
    null = null_summary(leave_one_out(variants))
    assert null["ok"], null
    for K in (4, 5, 6):
        for n in (6, 8, 11, 12, 14):
            neg = null_summary([null_row(b, runs[:K]) for b, runs in zip(bad[:n], variants[:n])])
            assert not neg["ok"], (K, n, neg)
            assert (neg["mean_u_min"] > NULL_U_MIN_FLOOR) == (n >= 11), (K, n, neg["mean_u_min"])
        assert null_summary(leave_one_out([runs[:K + 1] for runs in variants]))["ok"], K
