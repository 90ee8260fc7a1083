"""StableIdentification at block sizes other than the fixture's d = 5 (SURVEY A13 asks for "fixture
d = 5, then a scaled d"; coordinator.py:34-46 reads d from dim.csv): d = 8, the one-wave kernel's
limit, and d = 12 / 16, the multi-wave kernel (one thread per element of a d x d block: 192 / 256
threads, workgroup reductions, Gauss-Jordan / Cholesky / Jacobi on the whole workgroup;
csrc/riptrm_si.hip).  The instances follow the reference's dataset recipe
(oracle/si_oracle.py::synthetic_instance after src/StableIdentification/generator.py:18-134; its one
deviation — constraint values drawn around the start instead of an RALM-found interior start — is
documented there).  No reference output exists at these sizes: parity unpinned; the bar is the
fixture's (tests/test_gpu_si.py): HwCur 1e-12, teacher-forced tCG with the same stop and j, and
trajectories through parity.compare_until_flip."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from oracle import riptrm_oracle as RO
from oracle import si_oracle as SI

DS = (8, 12, 16)


def _inst(d, starts):
    return SI.synthetic_instance(d, 100 + d, starts=starts)


def _batch(data, B, cap=1024):
    import si
    eng = si.SIBatch(data.d, data.N, data.m, B, log_capacity=cap)
    eng.load(data.X, data.XP, data.h, np.asarray(data.cons, dtype=np.float64))
    return eng


@pytest.mark.parametrize("d", DS)
def test_si_scaled_hvp_matches_oracle(d):
    data, st = _inst(d, 4)
    B = len(st)
    xs = np.stack([x for x, _ in st])
    rs = np.random.RandomState(d)
    ys = np.stack([y for _, y in st]) * (0.5 + rs.rand(B, data.m))
    P = SI.SIVectorized(data)
    vs = np.stack([P.manifold.projection(xs[b], rs.randn(3, d, d)) for b in range(B)])
    mus = np.array([0.1, 1e-3, 1e-6, 0.02])
    out = _batch(data, B).hvp(xs, ys, mus, vs).cpu().numpy()
    for b in range(B):
        _, _, Hw, _ = P.begin_inner(xs[b], ys[b], mus[b])
        ref = Hw(vs[b])
        err = np.linalg.norm(out[b] - ref) / np.linalg.norm(ref)
        assert err < 1e-12, (d, b, err)
    Ps = SI.SIStructured(data)   # and the reference-structured wiring
    _, _, Hw, _ = Ps.begin_inner(xs[0], ys[0], mus[0])
    ref = Hw(vs[0])
    assert np.linalg.norm(out[0] - ref) / np.linalg.norm(ref) < 1e-12


@pytest.mark.parametrize("d", DS)
def test_si_scaled_tcg_teacher_forced(d):
    """Same (x, y, mu, Delta) in -> the same tCG stop reason, the same exit index j for short runs
    (long CG runs' exit index is a rounding quantity: within 1% there), eta within 1e-8."""
    data, st = _inst(d, 6)
    B = len(st)
    xs = np.stack([x for x, _ in st])
    ys = np.stack([y for _, y in st])
    rs = np.random.RandomState(7 + d)
    P = SI.SIVectorized(data)
    mus = np.array([0.1, 0.01, 1e-4, 0.1, 0.01, 1e-4])
    deltas = np.array([P.manifold.typical_dist / 8, 0.05, 0.2, 1e-3, 1.0, 0.01])
    ys = ys * (0.5 + rs.rand(B, data.m))
    eta, _, js, stops = _batch(data, B).tcg(xs, ys, mus, deltas)
    eta = eta.cpu().numpy()
    for b in range(B):
        _, _, Hw, c = P.begin_inner(xs[b], ys[b], mus[b])
        e, _, j, stop = RO.truncated_conjugate_gradient(P.manifold, Hw, xs[b], c, deltas[b], 1, 0.1, 1, P.manifold.dim)
        assert stops[b] == stop, (d, b, stops[b], stop, js[b], j)
        if j < 50:
            assert js[b] == j, (d, b, js[b], j)
        assert abs(int(js[b]) - j) <= max(2, 0.01 * j), (d, b, js[b], j)
        err = np.linalg.norm(eta[b] - e) / max(np.linalg.norm(e), 1e-300)
        assert err <= 1e-8, (d, b, j, err)


# (d, starts, maxiter): windows whose outer iterations all converge (inner_maxiter None, the
# reference's default), so the final x, y are real iterates -- no inner_maxiter reset to the outer
# step's start point (RIPTRM.py:835-842).  Measured on the oracle: d = 8 converges its first two
# outer iterations in 116-145 and 21-31 inner iterations, d = 12 / 16 their first in 510-1510 /
# 1420-1670 (~10 s / ~85-150 s per oracle run).
SI_WINDOWS = [(16, 3, 1), (12, 3, 1), (8, 6, 2)]


@pytest.mark.timeout(900)
def test_si_scaled_trajectory_matches_oracle(capsys):
    """At d = 8 (six starts, two outer iterations), 12 and 16 (three starts, one outer iteration
    each), twelve instances pooled into one rank test, every outer iteration run to its inner
    convergence test (SI_WINDOWS), under the null-calibrated bar (tests/parity.py check_null /
    assert_null; RIPTRM.py:574-629, 631-705, 785-976): these trajectories amplify rounding fast
    (at d = 12 two CPU back-ends with identical branches are 2e-5 apart in the cost and 60% in the
    residual by row 13, and their first branch flip comes after 9-50 rows), so the GPU is compared
    row by row only where the reference run is reproducible under summation order -- before every
    order variant's first flip (parity.si_variant: the reference-structured wiring at d = 8, where it
    finishes in seconds, and coordinate / constraint-order permutations) and before its own -- and
    over the whole window it must leave the reference run like one more such variant: final x, y
    and the outer iterates' KKT residuals within the gross bar, its divergence row, dx, dy and outer
    deviation ranked among the variants' as an exchangeable run would be.  Every variant must end
    away from the reference run (dx, dy > 0): the final-point statistics are not vacuous."""
    import si
    from parity import assert_null, check_si_parallel
    items = []
    for d, starts, maxiter in SI_WINDOWS:
        opt = {"maxiter": maxiter, "inner_maxiter": None, "tolresid": 0.0, "maxtime": 1e9}
        data, st = _inst(d, starts)
        xs = np.stack([x for x, _ in st])
        ys = np.stack([y for _, y in st])
        res = _batch(data, len(st), cap=4096).solve(xs, ys, dict(opt, TRS_solver="tCG", second_order_stationarity=False,
                                                                 manviofun=si.si_manviofun))
        gx, gy = res.x.cpu().numpy(), res.y.cpu().numpy()
        for b in range(len(st)):
            gl = res.log(b)
            assert int(res.stats[b, _C("OUTER_ITERS")]) == maxiter
            conv = [s_ for s_ in gl["inner_status"] if s_ == "converged"]
            assert len(conv) == maxiter, (d, b, "every outer iteration ends converged")
            items.append(dict(data=data, x0=xs[b], y0=ys[b], opt=opt, gl=gl, gpu_x=gx[b].reshape(3, d, d),
                              gpu_y=gy[b][:data.m], variants=(["structured", 1, 2, 3] if d == 8 else [1, 2, 3, 4]),
                              name=f"d={d} start {b}"))
        print(f"[si null] d={d}: GPU solve of {len(st)} starts done", flush=True)
    with capsys.disabled():
        results = check_si_parallel(items, progress=lambda m: print(m, flush=True))
        names = [it["name"] for it in items]
        for it in items:   # the starting point's KKT residual: the same formula on the same data
            r0 = results[it["name"]]["ref_residual0"]
            assert abs(it["gl"]["residual"][0] - r0) <= 1e-12 * r0, it["name"]
        assert_null([results[nm] for nm in names], names, _table("si_scaled"), variants_move=True)


def _C(name):
    from engine import C
    return C[f"RIPTRM_STAT_{name}"]


def _table(name):
    import os
    return os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out", "parity", name + ".json")


@pytest.mark.timeout(600)
@pytest.mark.parametrize("d,sos,inner", [(8, True, 6), (16, False, 2)])
def test_si_scaled_exact_repmat_hbm(d, sos, inner):
    """TRS_solver = 'Exact_RepMat' past d = 7 (RIPTRM.py:433-444, :599-617 with TRSgep :218-299):
    manifold.dim = 100 (d = 8) / 392 (d = 16) > RIPTRM_TRS_DIM_MAX, so each instance builds the matrix
    of HwCur (manifold.dim HVPs) in HBM and parks; riptrm_si_solve serves the parked instances in
    batched passes of the NonnegPCA HBM service (d = 8: the hand-written eigensolver of riptrm_eig.h and
    SciPy's CG in its eigen-coordinates; d = 16: the distributed tridiagonalisation of riptrm_tri.h and
    the subproblem in T's coordinates; the secular solve) and relaunches.  Bars: an instance's trajectory is bitwise the one it has solved alone (a slot's
    arithmetic does not depend on its pass), and each instance's rows meet compare_until_flip's bar
    against the oracle (trs_oracle: the reference's 2n x 2n pencil).  One outer iteration with a
    few inner ones: the oracle's own cost at these sizes (~2 s per inner iteration at d = 8 with the
    second-order test, ~14 s at d = 16) bounds the window."""
    import si
    from parity import compare_until_flip
    data, st = _inst(d, 2)
    xs = np.stack([x for x, _ in st])
    ys = np.stack([y for _, y in st])
    opt = {"maxiter": 1, "inner_maxiter": inner, "tolresid": 0.0, "maxtime": 1e9, "TRS_solver": "Exact_RepMat",
           "second_order_stationarity": sos}
    res = _batch(data, 2).solve(xs, ys, dict(opt, manviofun=si.si_manviofun))
    alone = _batch(data, 1).solve(xs[1:], ys[1:], dict(opt, manviofun=si.si_manviofun))
    for key in ("cost", "residual", "normdx", "mineigvalHw", "dxtype"):
        assert res.log(1)[key] == alone.log(0)[key], key
    np.testing.assert_array_equal(res.x[1].cpu().numpy(), alone.x[0].cpu().numpy())
    for b in range(2):
        gl = res.log(b)
        kinds = [k for k in gl["dxtype"] if k is not None]
        assert 0 < len(kinds) <= inner and all(k in ("boundary", "interior", "hardcase_1") for k in kinds), kinds
        assert (len([v for v in gl["mineigvalHw"] if v is not None]) > 0) == sos
        ref = SI.solve(data, xs[b], ys[b], dict(opt, manviofun=SI.si_manvio))
        compare_until_flip(gl, ref.log)


@pytest.mark.timeout(600)
def test_si_exact_hbm_eigensolve_failure_stops_one_instance():
    """bench.si_starts' start 30 at d = 8 drives the subproblem's eigensolve to non-convergence
    within two outer iterations -- on the CPU as well: there the oracle's scipy.linalg.eig raises
    LinAlgError (LAPACK ggev info 111) on the reference's pencil.  The reference's do_exit_on_error
    break (RIPTRM.py:961-966) ends that run with the iterate its outer step started from; the device
    stops only that instance (stats.error = RIPTRM_ERR_EIGEN), and the healthy instance of the same
    batch is bitwise the one solved alone."""
    import bench
    import si
    from engine import C
    xs, ys, (X, XP, h, constset) = bench.si_starts(2, [30, 1], 8)
    cons = si.expand_constset(constset)
    opt = {"maxiter": 2, "tolresid": 0.0, "maxtime": 1e9, "TRS_solver": "Exact_RepMat",
           "second_order_stationarity": True, "manviofun": si.si_manviofun}

    def run(sel):
        eng = si.SIBatch(8, X.shape[1], cons.shape[0], len(sel), log_capacity=1024)
        eng.load(X, XP, h, cons)
        return eng.solve(xs[sel], ys[sel], opt)

    both, alone = run([0, 1]), run([1])
    assert int(both.stats[0, C["RIPTRM_STAT_ERROR"]]) == C["RIPTRM_ERR_EIGEN"]
    assert int(both.stats[1, C["RIPTRM_STAT_ERROR"]]) == C["RIPTRM_ERR_NONE"]
    assert np.all(np.isfinite(both.x[0].cpu().numpy()))
    for key in ("cost", "residual", "normdx", "mineigvalHw"):
        assert both.log(1)[key] == alone.log(0)[key], key
    np.testing.assert_array_equal(both.x[1].cpu().numpy(), alone.x[0].cpu().numpy())


@pytest.mark.timeout(600)
def test_si_exact_hbm_many_columns():
    """k_si_repmat keeps each workgroup's residual E = XP - (I + hA) X (d x N) in LDS while d N 8 <=
    48 KiB and in its own slice of an HBM scratch beyond: d = 8 with the data columns replicated to
    N = 855 takes the HBM slices.  Bar: the oracle's (compare_until_flip), as for the LDS case."""
    import si
    from parity import compare_until_flip
    import copy
    base, st = _inst(8, 1)
    data = copy.copy(base)
    data.X, data.XP = np.tile(base.X, (1, 9)), np.tile(base.XP, (1, 9))
    data.N = data.X.shape[1]
    assert data.N * 8 * 8 > 48 * 1024
    xs = np.stack([x for x, _ in st])
    ys = np.stack([y for _, y in st])
    opt = {"maxiter": 1, "inner_maxiter": 3, "tolresid": 0.0, "maxtime": 1e9, "TRS_solver": "Exact_RepMat",
           "second_order_stationarity": False}
    res = _batch(data, 1).solve(xs, ys, dict(opt, manviofun=si.si_manviofun))
    ref = SI.solve(data, xs[0], ys[0], dict(opt, manviofun=SI.si_manvio))
    gl = res.log(0)
    assert 0 < len([k for k in gl["dxtype"] if k is not None]) <= 3
    compare_until_flip(gl, ref.log)


@pytest.mark.timeout(600)
@pytest.mark.parametrize("d,sos,bench_starts", [(8, True, True), (8, False, False), (16, True, False)])
def test_si_exact_cg_skip_is_bitwise_neutral(d, sos, bench_starts, monkeypatch):
    """The StableIdentification HBM service decides on the eigenpairs whether SciPy's CG
    (RIPTRM.py:246-251) can matter: it skips the CG only where a bound from them shows no CG iterate
    that passes the reference's residual / radius test can have p1obj <= xobj (RIPTRM.py:294-298;
    riptrm_trs_big.hip k_cg_wg).  So the default and RIPTRM_CG_SKIP=0 (always run the CG, in the
    order the NonnegPCA path uses) must give the same logs (cost, residual, normdx, dxtype,
    mineigvalHw) and x / y bit for bit; on the bench's own d = 8 starts some CGs must really be
    skipped (the test is not vacuous)."""
    import bench
    import si
    if bench_starts:
        xs, ys, (X, XP, h, constset) = bench.si_starts(8, list(range(8)), d)
        cons = si.expand_constset(constset)
        mk = lambda: _load(si.SIBatch(d, X.shape[1], cons.shape[0], len(xs), log_capacity=1024), X, XP, h, cons)   # noqa: E731
        opt = {"maxiter": 3, "tolresid": 0.0, "maxtime": 1e9}
    else:
        data, st = _inst(d, 2)
        xs = np.stack([x for x, _ in st])
        ys = np.stack([y for _, y in st])
        mk = lambda: _batch(data, len(xs))   # noqa: E731
        opt = {"maxiter": 1, "inner_maxiter": 4, "tolresid": 0.0, "maxtime": 1e9}
    opt.update(TRS_solver="Exact_RepMat", second_order_stationarity=sos, manviofun=si.si_manviofun)
    monkeypatch.delenv("RIPTRM_CG_SKIP", raising=False)
    e1 = mk()
    r1 = e1.solve(xs, ys, opt)
    checked, skipped = e1.trs_skip_stats()
    monkeypatch.setenv("RIPTRM_CG_SKIP", "0")
    e0 = mk()
    r0 = e0.solve(xs, ys, opt)
    assert e0.trs_skip_stats() == (0, 0)
    print(f"d={d} sos={sos}: {checked} subproblems decided on their eigenpairs, {skipped} CGs skipped")
    # manifold.dim 100 (d = 8) runs the one-workgroup CG, where the skip is decided on the
    # eigenpairs; 392 (d = 16) the tridiagonal path, where k_tri_solve decides it on T
    assert checked > 0, checked
    if bench_starts:
        assert skipped > 0
    for b in range(len(xs)):
        for key in ("cost", "residual", "normdx", "dxtype", "mineigvalHw", "inner_status", "radius_update"):
            assert r1.log(b)[key] == r0.log(b)[key], (b, key)
    np.testing.assert_array_equal(r1.x.cpu().numpy(), r0.x.cpu().numpy())
    np.testing.assert_array_equal(r1.y.cpu().numpy(), r0.y.cpu().numpy())


@pytest.mark.timeout(600)
@pytest.mark.parametrize("sos", [True, False])
def test_si_exact_eigen_cache_is_bitwise_neutral(sos, monkeypatch):
    """The SI service's keyed eigendecomposition cache (riptrm_si_solve, KeyedEigCache): a subproblem
    parked at exactly the point of the trial eigen-test before it (accepted step, no dual clipping,
    same mu) takes that eigensolve's compact eigenpairs and builds no matrix, as RIPTRM.py:686-692
    reuses HwNewmatrix.  The matrix would be the same bits, so RIPTRM_SI_CACHE=1 (opt-in: the
    lock-step service is pass-latency-bound) and the default must give the same logs and
    x / y bit for bit; with the second-order test the bench's d = 8 starts must really hit (the test
    is not vacuous)."""
    import bench
    import si
    d = 8
    xs, ys, (X, XP, h, constset) = bench.si_starts(8, list(range(8)), d)
    cons = si.expand_constset(constset)
    mk = lambda: _load(si.SIBatch(d, X.shape[1], cons.shape[0], len(xs), log_capacity=1024), X, XP, h, cons)   # noqa: E731
    opt = {"maxiter": 3, "tolresid": 0.0, "maxtime": 1e9, "TRS_solver": "Exact_RepMat",
           "second_order_stationarity": sos, "manviofun": si.si_manviofun}
    monkeypatch.setenv("RIPTRM_SI_CACHE", "1")
    e1 = mk()
    r1 = e1.solve(xs, ys, opt)
    hits, subs = e1.trs_cache_stats()
    monkeypatch.setenv("RIPTRM_SI_CACHE", "0")
    e0 = mk()
    r0 = e0.solve(xs, ys, opt)
    assert e0.trs_cache_stats()[0] == 0
    print(f"sos={sos}: {hits} of {subs} subproblems served from the cache")
    assert subs > 0
    assert (hits > 0) == sos, hits   # without the second-order test there is no trial eigensolve to keep
    for b in range(len(xs)):
        for key in ("cost", "residual", "normdx", "dxtype", "mineigvalHw", "inner_status", "radius_update"):
            assert r1.log(b)[key] == r0.log(b)[key], (b, key)
    np.testing.assert_array_equal(r1.x.cpu().numpy(), r0.x.cpu().numpy())
    np.testing.assert_array_equal(r1.y.cpu().numpy(), r0.y.cpu().numpy())


@pytest.mark.timeout(600)
def test_si_exact_prep_records_are_bitwise_neutral(monkeypatch):
    """k_si_prep computes each parked instance's prepare / frame / X X^T once and the matrix's column
    workgroups load them (RIPTRM.py:720-730 at the park point); RIPTRM_SI_PREP=0 has every workgroup
    recompute them.  The same code on the same inputs: logs and x / y bit for bit."""
    import bench
    import si
    d = 8
    xs, ys, (X, XP, h, constset) = bench.si_starts(8, list(range(8)), d)
    cons = si.expand_constset(constset)
    mk = lambda: _load(si.SIBatch(d, X.shape[1], cons.shape[0], len(xs), log_capacity=1024), X, XP, h, cons)   # noqa: E731
    opt = {"maxiter": 2, "tolresid": 0.0, "maxtime": 1e9, "TRS_solver": "Exact_RepMat",
           "second_order_stationarity": True, "manviofun": si.si_manviofun}
    monkeypatch.delenv("RIPTRM_SI_PREP", raising=False)
    r1 = mk().solve(xs, ys, opt)
    monkeypatch.setenv("RIPTRM_SI_PREP", "0")
    r0 = mk().solve(xs, ys, opt)
    for b in range(len(xs)):
        for key in ("cost", "residual", "normdx", "dxtype", "mineigvalHw", "inner_status", "radius_update"):
            assert r1.log(b)[key] == r0.log(b)[key], (b, key)
    np.testing.assert_array_equal(r1.x.cpu().numpy(), r0.x.cpu().numpy())
    np.testing.assert_array_equal(r1.y.cpu().numpy(), r0.y.cpu().numpy())


def _load(eng, X, XP, h, cons):
    eng.load(X, XP, h, cons)
    return eng
