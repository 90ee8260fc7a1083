"""GPU parity tests: the HIP path (through the C-ABI) against the CPU oracle on the same inputs.

Tolerances (fp64 throughout; the only differences are reduction order and libm-vs-ocml log/acos):
* operator level (S-pass, barrier Hessian, tCG step from the same state): rel 1e-12 / 1e-9;
* trajectory level (whole solve): identical branch decisions and per-row values within the
  bounds of tests/parity.py, calibrated on the two CPU oracles against each other
  (tests/test_oracle.py::test_comparator_calibration).
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from oracle import nonnegpca_gen as G
from oracle import riptrm_oracle as O

OPT = dict(tolresid=0.0, maxtime=1e9)


def _engine(Z, cap=4096, layout="sym", groups=0):
    """layout "sym2": the symmetric-tile layout with the super-tile S-pass forced (spass_kind 2)."""
    import engine
    Z = np.asarray(Z)
    if Z.ndim == 2:
        Z = Z[None]
    kind = 2 if layout == "sym2" else 1
    eng = engine.NonnegPCABatch(Z.shape[1], Z.shape[0], log_capacity=cap, layout=layout.rstrip("2"),
                                stream_groups=groups, spass_kind=kind)
    eng.load_Z(Z)
    return eng


def _gpu_opt(**kw):
    from problems import manviofun
    o = {"TRS_solver": "tCG", "second_order_stationarity": False, "manviofun": manviofun}
    o.update(OPT)
    o.update(kw)
    return o


def _oracle_opt(**kw):
    o = dict(OPT, manviofun=O.sphere_manvio)
    o.update(kw)
    return o


def _state(n, seed):
    rs = np.random.RandomState(seed)
    x = np.abs(rs.rand(n)) + 1e-3
    x /= np.linalg.norm(x)
    y = rs.rand(n) + 0.05
    return x, y


@pytest.mark.parametrize("layout", ["sym", "full"])
@pytest.mark.parametrize("n", [2, 17, 40, 50, 129, 333, 1000])
def test_pack_is_exact_symmetrization(n, layout):
    Z, _, _ = G.generate_instance(n, 3)
    Z2 = Z.T * 0.5
    eng = _engine(np.stack([Z, Z2]), layout=layout)
    np.testing.assert_array_equal(eng.unpack(0), Z + Z.T)          # exact: one add per element
    np.testing.assert_array_equal(eng.unpack(1), Z2 + Z2.T)
    S = eng.S.cpu().numpy()
    assert np.isfinite(S).all()
    if layout == "full":   # padding is zero
        full = S[0][: eng.rows * eng.ld].reshape(eng.rows, eng.ld)
        assert not full[n:, :].any() and not full[:, n:].any()


@pytest.mark.parametrize("layout", ["sym", "sym2", "full"])
@pytest.mark.parametrize("n,B", [(17, 3), (50, 2), (200, 2), (300, 3), (1000, 3), (4000, 2)])
def test_barrier_hessian_matches_oracle(n, B, layout):
    Zs, xs, ys, vs = [], [], [], []
    for b in range(B):
        Z, _, _ = G.generate_instance(n, 10 + b)
        x, y = _state(n, 20 + b)
        Zs.append(Z); xs.append(x); ys.append(y)
        vs.append(np.random.RandomState(30 + b).randn(n))
    eng = _engine(np.stack(Zs), layout=layout)
    mu = 0.0123
    out = eng.hvp(np.stack(xs), np.stack(ys), mu, np.stack(vs)).cpu().numpy()
    for b in range(B):
        P = O.NonnegPCAVectorized(Zs[b])
        _, _, Hw, _ = P.begin_inner(xs[b], ys[b], mu)
        ref = Hw(vs[b])
        err = np.linalg.norm(out[b] - ref) / np.linalg.norm(ref)
        assert err < 1e-12, (b, err)


@pytest.mark.parametrize("n", [50, 200, 1000])
def test_tcg_matches_oracle_teacher_forced(n):
    """Same (x, y, mu, Delta) in -> same tCG exit (stop reason, j) and eta."""
    B = 6
    Zs, xs, ys = [], [], []
    for b in range(B):
        Z, x0, y0 = G.generate_instance(n, 40 + b)
        Zs.append(Z); xs.append(x0); ys.append(y0)
    mus = np.array([0.1, 0.05, 1e-2, 1e-3, 0.1, 0.02])
    deltas = np.array([np.pi / 8, 1e-3, 0.05, 0.3, 5.0, 0.01])
    eng = _engine(np.stack(Zs))
    eta, heta, js, stops = eng.tcg(np.stack(xs), np.stack(ys), mus, deltas)
    eta = eta.cpu().numpy()
    heta = heta.cpu().numpy()
    for b in range(B):
        P = O.NonnegPCAVectorized(Zs[b])
        _, _, Hw, c = P.begin_inner(xs[b], ys[b], mus[b])
        e, he, j, stop = O.truncated_conjugate_gradient(P.manifold, Hw, xs[b], c, deltas[b], 1, 0.1, 1, n - 1)
        assert stops[b] == stop, (b, stops[b], stop)
        assert js[b] == j, (b, js[b], j)
        assert np.linalg.norm(eta[b] - e) <= 1e-9 * max(np.linalg.norm(e), 1e-300), b
        assert np.linalg.norm(heta[b] - he) <= 1e-8 * max(np.linalg.norm(he), 1e-300), b


def _compare_logs(gl, rl):
    from parity import compare_logs
    compare_logs(gl, rl)


def test_full_solve_fixture_n50(fixture_n50):
    from problems import NonnegPCAProblem
    from RIPTRM import RIPTRM
    Z, x0, y0 = fixture_n50
    out = RIPTRM(_gpu_opt(maxiter=12)).run(NonnegPCAProblem(Z=Z, initialpoint=x0, initialineqLagmult=y0))
    ref = O.solve(Z, x0, y0, _oracle_opt(maxiter=12))
    assert f"{out.log['residual'][0]:.6e}" == "4.986888e+00"
    _compare_logs(out.log, ref.log)
    np.testing.assert_allclose(out.x, ref.x, atol=1e-6)
    np.testing.assert_allclose(out.ineqLagmult, ref.y, rtol=1e-3, atol=1e-6)
    assert out.option["stoppingcriterion"].startswith("Max iteration count reached; maxiter=12 after")
    assert out.name == "RIPTRM_tCG"


def test_fixture_reaches_published_residual_on_gpu(fixture_n50):
    """analyzer.ipynb: RIPTRM (tCG) on dataset/NonnegPCA/1/a plateaus at ~1e-14."""
    from problems import NonnegPCAProblem
    from RIPTRM import RIPTRM
    Z, x0, y0 = fixture_n50
    out = RIPTRM(_gpu_opt(maxiter=45)).run(NonnegPCAProblem(Z=Z, initialpoint=x0, initialineqLagmult=y0))
    res = np.array(out.log["residual"], float)
    conv = [i for i, s in enumerate(out.log["inner_status"]) if s in (None, "converged")]
    assert res[conv][-1] < 2e-14


def _table(name):
    """Where a null test writes its per-instance table (merged back from the GPU box)."""
    import os
    return os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out", "parity", name + ".json")


def _null_pool(groups, name):
    """The null-calibrated bar (tests/parity.py check_null / assert_null) over the instances of all
    `groups` pooled into ONE rank test: groups = [(K, [item, ...]), ...] with the items of
    parity.check_instances_parallel (the six oracle runs of each instance on a pool of
    single-threaded processes).  A rank test over a handful of instances has no power (its mean-u
    limit is ~0 at 2-5 instances), so small-batch cases are judged together."""
    from parity import assert_null, check_instances_parallel
    rows, names = [], []
    for K, items in groups:
        res = check_instances_parallel(items, _oracle_opt(maxiter=K))
        for it in items:
            rows.append(res[it["name"]])
            names.append(it["name"])
    assert_null(rows, names, _table(name))


# (n, B, K, layout): 16 instances over sizes, layouts and S-pass kinds ("sym2": super-tile forced)
BATCHED_CASES = [(37, 5, 10, "sym"), (200, 4, 12, "sym"), (1000, 2, 10, "sym"), (300, 3, 10, "sym2"), (1000, 2, 10, "sym2")]


@pytest.mark.timeout(900)
def test_batched_solve_matches_oracle():
    """Per instance: the envelope bar row by row where the reference run is reproducible under
    summation order; over the whole window the null-calibrated bar, all 16 instances of the five
    batched solves (BATCHED_CASES) pooled into one rank test (tests/parity.py check_null /
    assert_null; RIPTRM.py:631-705, 785-976)."""
    groups = []
    for n, B, K, layout in BATCHED_CASES:
        insts = [G.generate_instance(n, 100 + b) for b in range(B)]
        eng = _engine(np.stack([z for z, _, _ in insts]), layout=layout)
        res = eng.solve(np.stack([x for _, x, _ in insts]), np.stack([y for _, _, y in insts]), _gpu_opt(maxiter=K))
        xs, ys = res.x.cpu().numpy(), res.y.cpu().numpy()
        items = []
        for b, (Z, x0, y0) in enumerate(insts):
            assert int(res.stat(b, "OUTER_ITERS")) == K
            items.append(dict(gl=res.log(b), S=Z + Z.T, x0=x0, y0=y0, gpu_x=xs[b][:n], gpu_y=ys[b][:n],
                              gpu_tcg=res.tcg_iters_per_row(b)[1:], name=f"n={n} {layout} instance {b}"))
        groups.append((K, items))
        print(f"[batched] n={n} B={B} {layout}: GPU solve done", flush=True)
    _null_pool(groups, "batched")


def test_edge_options_match_oracle():
    Z, x0, y0 = G.generate_instance(9, 7)
    cases = [dict(maxiter=0), dict(maxiter=4, tolresid=1e3), dict(maxiter=3, inner_maxiter=1),
             dict(maxiter=4, save_inner_iteration=False), dict(maxiter=3, initial_TR_radius=1e-4),
             dict(maxiter=5, do_simple_barrier_parameter_update=False)]
    for kw in cases:
        eng = _engine(Z)
        res = eng.solve(x0[None], y0[None], _gpu_opt(**kw))
        ref = O.solve(Z, x0, y0, _oracle_opt(**kw))
        _compare_logs(res.log(0), ref.log)
        gs, rs_ = (res.stopping_criterion(0) or ""), ref.stoppingcriterion
        if rs_.startswith("KKT residual tolerance reached"):
            assert gs.startswith("KKT residual tolerance reached; current residual="), kw
            gv = float(gs.split("residual=")[1].split(" ")[0])
            rv = float(rs_.split("residual=")[1].split(" ")[0])
            assert abs(gv - rv) <= 1e-12 * abs(rv), kw
        else:
            assert gs.split(" after")[0] == rs_.split(" after")[0], kw


def test_tiny_n2():
    Z, x0, y0 = G.generate_instance(2, 1)
    eng = _engine(Z)
    res = eng.solve(x0[None], y0[None], _gpu_opt(maxiter=6))
    ref = O.solve(Z, x0, y0, _oracle_opt(maxiter=6))
    _compare_logs(res.log(0), ref.log)


def test_pause_resume_is_transparent():
    """Stopping every instance at outer-iteration targets and resuming changes nothing."""
    n, B = 120, 3
    insts = [G.generate_instance(n, 300 + b) for b in range(B)]
    Z = np.stack([z for z, _, _ in insts])
    X0 = np.stack([x for _, x, _ in insts])
    Y0 = np.stack([y for _, _, y in insts])
    e1 = _engine(Z)
    r1 = e1.solve(X0, Y0, _gpu_opt(maxiter=9))
    e2 = _engine(Z)
    e2.begin(X0, Y0, _gpu_opt(maxiter=9))
    for tgt in (2, 5, 7, None):
        e2.run_until(tgt)
    r2 = e2.result()
    for b in range(B):
        a, c = r1.log(b), r2.log(b)
        for k in a:
            if k != "time":
                assert a[k] == c[k] or np.allclose(np.array(a[k], float), np.array(c[k], float), rtol=0, atol=0), k
    assert torch.equal(r1.x, r2.x)


def test_large_n4000_properties():
    """n = 4000 (BASELINE config 3's size): symmetric operator, tangent output, S-pass vs torch."""
    n = 4000
    Z, x0, y0 = G.generate_instance(n, 4242)
    eng = _engine(Z)
    S = torch.tensor(eng.unpack(0), device="cuda")
    rs = np.random.RandomState(1)
    x = x0
    y = rs.rand(n) + 0.1
    u = rs.randn(n); u -= (x @ u) * x
    v = rs.randn(n); v -= (x @ v) * x
    Hu = eng.hvp(x, y, 0.01, u).cpu().numpy()[0]
    Hv = eng.hvp(x, y, 0.01, v).cpu().numpy()[0]
    assert abs(u @ Hv - v @ Hu) <= 1e-10 * np.linalg.norm(Hu) * np.linalg.norm(v)
    P = O.NonnegPCAVectorized(Z)
    _, _, Hw, _ = P.begin_inner(x, y, 0.01)
    assert np.linalg.norm(Hu - Hw(u)) <= 1e-12 * np.linalg.norm(Hu)
    Sx = (S @ torch.tensor(x, device=S.device)).cpu().numpy()
    np.testing.assert_allclose(Sx, (Z + Z.T) @ x, rtol=1e-12, atol=1e-12)


def test_deterministic_and_batch_independent():
    """Fixed reduction orders: the same instance gives bit-identical iterates and logs whether it
    is solved alone, in a batch on one stream, or in a batch split over two stream groups."""
    n = 300
    insts = [G.generate_instance(n, 500 + b) for b in range(9)]
    Z = np.stack([z for z, _, _ in insts])
    X0 = np.stack([x for _, x, _ in insts])
    Y0 = np.stack([y for _, _, y in insts])
    r1 = _engine(Z, groups=2).solve(X0, Y0, _gpu_opt(maxiter=8))
    r2 = _engine(Z, groups=1).solve(X0, Y0, _gpu_opt(maxiter=8))
    r3 = _engine(Z[4:5]).solve(X0[4:5], Y0[4:5], _gpu_opt(maxiter=8))
    assert torch.equal(r1.x, r2.x) and torch.equal(r1.y, r2.y)
    assert torch.equal(r1.x[4:5], r3.x)
    for a, c in ((r1.log(4), r2.log(4)), (r1.log(4), r3.log(0))):
        for k in a:
            if k != "time":
                assert a[k] == c[k] or np.array_equal(np.array(a[k], float), np.array(c[k], float)), k


def test_simulator_end_to_end_fixture(tmp_path):
    """cfg -> coordinator -> RIPTRM on the GPU -> CSVs in the reference layout."""
    import os
    import shutil
    import pandas as pd
    from conftest import GOLDEN
    from simulator import Simulator
    ds = tmp_path / "dataset" / "NonnegPCA" / "1"
    ds.mkdir(parents=True)
    for f in ("dim.csv", "Z.csv", "initx_a.csv", "initineqLagmult.csv"):
        shutil.copy(os.path.join(GOLDEN, "nonnegpca_1", f), ds / f)
    cfg = {"problem_name": "NonnegPCA", "problem_instance": 1, "problem_initialpoint": "a",
           "problem_coordinator_name": "coordinator", "solver_name": ["RIPTRM"],
           "solver_option": {"common": {"maxtime": 240, "maxiter": 6, "tolresid": 1e-16, "verbosity": 0},
                             "RIPTRM": {"TRS_solver": "tCG", "second_order_stationarity": False}}}
    outs = Simulator(cfg, root=str(tmp_path)).run()
    d = tmp_path / "intermediate" / "NonnegPCA" / "1" / "a"
    log = pd.read_csv(d / "RIPTRM_tCG_log.csv")
    assert abs(log["residual"][0] - 4.986888432851817) < 1e-12
    assert log["iteration"].max() == 6
    assert np.allclose(np.loadtxt(d / "RIPTRM_tCG_x.csv"), outs[0].x)


# ---- shared layout (multi-start: one Z, many initial points; fp64 MFMA S-pass) ----------------

def _shared_engine(Z, B, cap=4096):
    import engine
    eng = engine.NonnegPCABatch(Z.shape[0], B, log_capacity=cap, layout="shared")
    eng.load_Z(Z)
    return eng


@pytest.mark.parametrize("n", [2, 37, 129, 1000])
def test_shared_pack_is_exact_symmetrization(n):
    Z, _, _ = G.generate_instance(n, 5)
    eng = _shared_engine(Z, 3)
    np.testing.assert_array_equal(eng.unpack(0), Z + Z.T)
    assert eng.S.shape[0] == 1


@pytest.mark.parametrize("n,B", [(17, 3), (50, 33), (200, 130), (1000, 40), (4000, 20)])
def test_shared_barrier_hessian_matches_oracle(n, B):
    """Both MFMA tilings (<= 32 and > 32 right-hand sides), ragged n and B."""
    Z, _, _ = G.generate_instance(n, 11)
    xs, ys, vs = [], [], []
    for b in range(B):
        x, y = _state(n, 200 + b)
        xs.append(x); ys.append(y)
        vs.append(np.random.RandomState(300 + b).randn(n))
    eng = _shared_engine(Z, B)
    mu = 0.0123
    out = eng.hvp(np.stack(xs), np.stack(ys), mu, np.stack(vs)).cpu().numpy()
    P = O.NonnegPCAVectorized(Z)
    for b in range(B):
        _, _, Hw, _ = P.begin_inner(xs[b], ys[b], mu)
        ref = Hw(vs[b])
        err = np.linalg.norm(out[b] - ref) / np.linalg.norm(ref)
        assert err < 1e-12, (b, err)


@pytest.mark.parametrize("n", [129, 1000, 4000])
def test_shared_product_independent_of_batch_bitwise(n):
    """k_spass_mm sums k in one order for every tile shape (128 or 32 right-hand sides per
    workgroup, 128- or 64-row tiles) and the K slices in slice order: an instance's Hessian
    action in a 40-wide batch equals, bit for bit, the same instance's in a 3-wide batch."""
    Z, _, _ = G.generate_instance(n, 13)
    B = 40
    xs, ys, vs = [], [], []
    for b in range(B):
        x, y = _state(n, 700 + b)
        xs.append(x); ys.append(y)
        vs.append(np.random.RandomState(800 + b).randn(n))
    xs, ys, vs = np.stack(xs), np.stack(ys), np.stack(vs)
    wide = _shared_engine(Z, B).hvp(xs, ys, 0.0123, vs)
    pick = [0, 17, 39]
    narrow = _shared_engine(Z, 3).hvp(xs[pick], ys[pick], 0.0123, vs[pick])
    assert torch.equal(wide[pick], narrow)


@pytest.mark.parametrize("n,B,K", [(200, 40, 8), (1000, 70, 5)])
def test_shared_solve_independent_of_batch_bitwise(n, B, K):
    """Whole multi-start solves: the passes where some starts ask for a second product (their
    in1 columns compacted into 32-wide tiles in list order) change no start's arithmetic, so
    three starts of a wide batch follow the same trajectory bit for bit when solved alone."""
    Z, _, y0 = G.generate_instance(n, 510)
    starts = []
    for b in range(B):
        x0 = np.abs(np.random.RandomState(900 + b).rand(n))
        starts.append(x0 / np.linalg.norm(x0))
    starts = np.stack(starts)
    ys = np.stack([y0] * B)
    wide = _shared_engine(Z, B).solve(starts, ys, _gpu_opt(maxiter=K))
    pick = [0, B // 2, B - 1]
    alone = _shared_engine(Z, 3).solve(starts[pick], ys[pick], _gpu_opt(maxiter=K))
    assert torch.equal(wide.x[pick], alone.x) and torch.equal(wide.y[pick], alone.y)
    for j, b in enumerate(pick):
        la, lb = wide.log(b), alone.log(j)
        for key in la:
            if key != "time":
                assert la[key] == lb[key] or np.array_equal(np.array(la[key], float), np.array(lb[key], float)), (b, key)


@pytest.mark.parametrize("n,B", [(200, 6), (1000, 36)])
def test_shared_tcg_matches_oracle_teacher_forced(n, B):
    Z, _, _ = G.generate_instance(n, 41)
    rs = np.random.RandomState(7)
    xs, ys = [], []
    for b in range(B):
        x, y = _state(n, 400 + b)
        xs.append(x); ys.append(y)
    mus = rs.choice([0.1, 0.05, 1e-2, 1e-3], B)
    deltas = rs.choice([np.pi / 8, 1e-3, 0.05, 0.3, 5.0], B)
    eng = _shared_engine(Z, B)
    eta, _, js, stops = eng.tcg(np.stack(xs), np.stack(ys), mus, deltas)
    eta = eta.cpu().numpy()
    P = O.NonnegPCAVectorized(Z)
    for b in range(B):
        _, _, Hw, c = P.begin_inner(xs[b], ys[b], mus[b])
        e, _, j, stop = O.truncated_conjugate_gradient(P.manifold, Hw, xs[b], c, deltas[b], 1, 0.1, 1, n - 1)
        assert stops[b] == stop and js[b] == j, (b, stops[b], stop, js[b], j)
        # the MFMA product sums k in another order than dsymv (permuted 32-chunks, 4 K slices);
        # CG amplifies that rounding over j iterations: 1e-8 here vs 1e-9 for the mat-vec layouts
        err = np.linalg.norm(eta[b] - e) / max(np.linalg.norm(e), 1e-300)
        assert err <= 1e-8, (b, j, err)


@pytest.mark.timeout(900)
@pytest.mark.parametrize("n,B,K", [(60, 40, 10), (1000, 12, 8)])
def test_shared_multistart_solve_matches_oracle(n, B, K):
    """One Z, B feasible starts (the MFMA shared-S layout): every start's trajectory against the
    oracle's under the null-calibrated bar, all B starts in one rank test (12 at n = 1000, so the
    test has power: tests/parity.py assert_null)."""
    Z, _, y0 = G.generate_instance(n, 500)
    starts = []
    for b in range(B):
        x0 = np.abs(np.random.RandomState(600 + b).rand(n))
        starts.append(x0 / np.linalg.norm(x0))
    eng = _shared_engine(Z, B)
    res = eng.solve(np.stack(starts), np.stack([y0] * B), _gpu_opt(maxiter=K))
    xs, ys = res.x.cpu().numpy(), res.y.cpu().numpy()
    S = Z + Z.T
    items = [dict(gl=res.log(b), S=S, x0=starts[b], y0=y0, gpu_x=xs[b][:n], gpu_y=ys[b][:n],
                  gpu_tcg=res.tcg_iters_per_row(b)[1:], name=f"start {b}") for b in range(B)]
    _null_pool([(K, items)], f"multistart_n{n}")


def test_run_batch_detects_shared_Z(fixture_n50):
    """problem_initialpoint axis: problems that share Z run on one shared S."""
    from problems import NonnegPCAProblem
    from RIPTRM import RIPTRM
    Z, x0, y0 = fixture_n50
    x1 = np.abs(np.random.RandomState(1).rand(Z.shape[0]))
    x1 /= np.linalg.norm(x1)
    solver = RIPTRM(_gpu_opt(maxiter=6))
    outs = solver.run_batch([NonnegPCAProblem(Z=Z, initialpoint=x0, initialineqLagmult=y0),
                             NonnegPCAProblem(Z=Z, initialpoint=x1, initialineqLagmult=y0)])
    assert solver.last_layout == "shared"
    single = RIPTRM(_gpu_opt(maxiter=6)).run(NonnegPCAProblem(Z=Z, initialpoint=x0, initialineqLagmult=y0))
    np.testing.assert_allclose(outs[0].log["residual"], single.log["residual"], rtol=1e-6, atol=1e-13)


@pytest.mark.parametrize("layout", ["sym", "sym2", "full"])
@pytest.mark.parametrize("n,B", [(23, 3), (1000, 2), (4000, 2)])
def test_ripm_operator_aw_matches_oracle(n, B, layout):
    """RIPM OperatorAw (RIPM.py:485-487) through the same S-pass as HwCur."""
    Zs, xs, zs, ss, vs = [], [], [], [], []
    for b in range(B):
        Z, _, _ = G.generate_instance(n, 60 + b)
        x, _ = _state(n, 70 + b)
        rs = np.random.RandomState(80 + b)
        Zs.append(Z); xs.append(x); zs.append(rs.rand(n) + 0.1); ss.append(rs.rand(n) + 0.2)
        vs.append(rs.randn(n))
    eng = _engine(np.stack(Zs), layout=layout)
    out = eng.operator_aw(np.stack(xs), np.stack(zs), np.stack(ss), np.stack(vs)).cpu().numpy()
    for b in range(B):
        ref = O.ripm_operator_aw_vectorized(Zs[b], xs[b], zs[b], ss[b], vs[b])
        assert np.linalg.norm(out[b] - ref) <= 1e-12 * np.linalg.norm(ref), b
    if n <= 100:   # the reference's per-constraint wiring too
        P = O.NonnegPCAStructured(Zs[0])
        ref = O.ripm_operator_aw(P, xs[0], zs[0], ss[0], vs[0])
        assert np.linalg.norm(out[0] - ref) <= 1e-12 * np.linalg.norm(ref)


@pytest.mark.parametrize("sos", [True, False])
@pytest.mark.parametrize("layout", ["sym", "sym2", "full"])
def test_exact_repmat_fixture_n50_matches_oracle(fixture_n50, sos, layout):
    """TRS_solver = 'Exact_RepMat' (RIPTRM.py:433-444) on dataset/NonnegPCA/1 point a: HwCur's
    matrix in the Householder frame of x^perp, TRSgep on the device (csrc/riptrm_trs.h), and with
    second_order_stationarity the eigen-check at every trial point (RIPTRM.py:599-617), against the
    oracle (the reference's 2n x 2n pencil, trs_oracle.trs_gep).  Same trajectory bar as tCG."""
    from parity import compare_until_flip
    Z, x0, y0 = fixture_n50
    K = 6
    opt = dict(TRS_solver="Exact_RepMat", second_order_stationarity=sos, maxiter=K)
    eng = _engine(Z, layout=layout)
    res = eng.solve(x0[None], y0[None], _gpu_opt(**opt))
    ref = O.solve(Z, x0, y0, _oracle_opt(**opt))
    gl = res.log(0)
    assert f"{gl['residual'][0]:.6e}" == "4.986888e+00"
    kinds = [k for k in gl["dxtype"] if k is not None]
    assert kinds and all(k in ("boundary", "interior", "hardcase_1") for k in kinds), kinds
    assert any(v is not None for v in gl["mineigvalHw"]) == sos
    compare_until_flip(gl, ref.log)


def test_exact_repmat_batch_matches_oracle():
    """A batch of instances (n = 33) with the class defaults (Exact_RepMat + second-order test)."""
    from parity import compare_until_flip
    insts = [G.generate_instance(33, 300 + b) for b in range(3)]
    eng = _engine(np.stack([z for z, _, _ in insts]))
    opt = dict(TRS_solver="Exact_RepMat", second_order_stationarity=True, maxiter=8)
    res = eng.solve(np.stack([x for _, x, _ in insts]), np.stack([y for _, _, y in insts]), _gpu_opt(**opt))
    for b, (Z, x0, y0) in enumerate(insts):
        compare_until_flip(res.log(b), O.solve(Z, x0, y0, _oracle_opt(**opt)).log)


def test_exact_repmat_reference_defaults_drop_in(fixture_n50):
    """RIPTRM(option) without TRS_solver runs the class default Exact_RepMat (RIPTRM.py:325), in
    LDS at n = 50 and on the HBM path at n = 120 (manifold.dim 119 > RIPTRM_TRS_DIM_MAX)."""
    from problems import NonnegPCAProblem, manviofun
    from RIPTRM import RIPTRM
    Z, x0, y0 = fixture_n50
    out = RIPTRM({"maxiter": 3, "tolresid": 0.0, "maxtime": 1e9, "manviofun": manviofun}).run(
        NonnegPCAProblem(Z=Z, initialpoint=x0, initialineqLagmult=y0))
    assert out.name == "RIPTRM_Exact_RepMat"
    assert any(v is not None for v in out.log["mineigvalHw"])
    Zb, xb, yb = G.generate_instance(120, 1)
    ob = RIPTRM({"maxiter": 2, "tolresid": 0.0, "maxtime": 1e9, "manviofun": manviofun}).run(
        NonnegPCAProblem(Z=Zb, initialpoint=xb, initialineqLagmult=yb))
    assert ob.name == "RIPTRM_Exact_RepMat" and max(ob.log["iteration"]) == 2
    assert any(v is not None for v in ob.log["mineigvalHw"])


@pytest.mark.timeout(600)
@pytest.mark.parametrize("n", [130, 200, 260])
@pytest.mark.parametrize("sos", [True, False])
def test_exact_repmat_above_lds_size_matches_oracle(sos, n):
    """NonnegPCA n = 130 / 200 / 260 (manifold.dim 129 / 199 / 259) with Exact_RepMat: the HBM path (frame
    matrix densified from S; at 129 the hand-written eigensolver and the CG in its eigen-coordinates, from
    150 on (RIPTRM_TRS_TRI_MIN) the distributed tridiagonalisation and the subproblem in T's coordinates, riptrm_tri.h; the
    trial-point eigenvalue with the second-order test) against the oracle (the reference's 2n x 2n
    pencil per inner step, trs_oracle.trs_gep; its per-constraint HVPs build the matrix), with the
    Exact_RepMat trajectory bar (parity.compare_until_flip)."""
    from parity import compare_until_flip
    Z, x0, y0 = G.generate_instance(n, 77)
    opt = dict(TRS_solver="Exact_RepMat", second_order_stationarity=sos, maxiter=4)
    eng = _engine(Z)
    res = eng.solve(x0[None], y0[None], _gpu_opt(**opt))
    ref = O.solve(Z, x0, y0, _oracle_opt(**opt))
    gl = res.log(0)
    kinds = [k for k in gl["dxtype"] if k is not None]
    assert kinds and all(k in ("boundary", "interior", "hardcase_1") for k in kinds), kinds
    assert any(v is not None for v in gl["mineigvalHw"]) == sos
    compare_until_flip(gl, ref.log)


@pytest.mark.timeout(600)
def test_exact_repmat_lds_and_hbm_paths_agree_near_97(monkeypatch):
    """the two Exact_RepMat paths at the size where they meet.  n = 97 (manifold.dim 96,
    the LDS solver's limit: Householder frame matrix, parallel Jacobi in LDS) solved again with
    RIPTRM_TRS_HBM=1 (the HBM service: densified frame matrix, coef = -x^T (M x) + y^T x in
    k_repmat_vec, the hand-written eigensolver of riptrm_eig.h with SciPy's CG in its eigen-coordinates
    (k_cg_diag), the eigenpair cache) -- the same reference step (RIPTRM.py:433-444,
    599-617, TRSgep :218-299) in two arithmetics, so their trajectories must agree with the bar the
    solo Exact test uses against the oracle (parity.compare_until_flip), and both against the oracle."""
    from parity import compare_until_flip
    Z, x0, y0 = G.generate_instance(97, 78)
    opt = dict(TRS_solver="Exact_RepMat", second_order_stationarity=True, maxiter=4)
    monkeypatch.delenv("RIPTRM_TRS_HBM", raising=False)
    lds = _engine(Z).solve(x0[None], y0[None], _gpu_opt(**opt))
    monkeypatch.setenv("RIPTRM_TRS_HBM", "1")
    e = _engine(Z)
    hbm = e.solve(x0[None], y0[None], _gpu_opt(**opt))
    assert e.trs_cache_stats()[1] > 0   # the HBM service really served the subproblems
    ref = O.solve(Z, x0, y0, _oracle_opt(**opt))
    for gl in (lds.log(0), hbm.log(0)):
        kinds = [k for k in gl["dxtype"] if k is not None]
        assert kinds and all(k in ("boundary", "interior", "hardcase_1") for k in kinds), kinds
        compare_until_flip(gl, ref.log)
    compare_until_flip(hbm.log(0), lds.log(0))


@pytest.mark.timeout(600)
@pytest.mark.parametrize("n", [130, 260])
def test_exact_repmat_above_lds_size_batched(monkeypatch, n):
    """The HBM Exact_RepMat service over a batch (csrc/riptrm_trs_big.hip: every parked instance in
    one pass, one workspace slot each; n = 130 the batched hand-written eigensolver, n = 260 the
    distributed tridiagonalisation, several matrices per cooperative launch): six instances with the
    second-order test.  Each instance's trajectory is the one it has solved alone (a slot's arithmetic does not
    depend on the pass it shares), whichever CG form serves it (one workgroup per slot or the
    grid-wide launches: the same sums in the same order), however many slots the scratch budget
    allows (one slot: six passes) and whether the eigendecomposition cache serves the subproblems at
    an accepted trial point (riptrm_trs_bind_cache: same matrix bits, so the same eigenpairs);
    instance 0 also meets the oracle bar of the solo test above."""
    from parity import compare_until_flip
    B, K = 6, 3
    insts = [G.generate_instance(n, 90 + b) for b in range(B)]
    Zs = np.stack([z for z, _, _ in insts])
    xs = np.stack([x for _, x, _ in insts])
    ys = np.stack([y for _, _, y in insts])
    opt = _gpu_opt(TRS_solver="Exact_RepMat", second_order_stationarity=True, maxiter=K)

    stats = {}

    def run(Z, x, y, cg=None, gb=None, cache=None):
        if cache:
            monkeypatch.setenv("RIPTRM_TRS_CACHE", cache)
        else:
            monkeypatch.delenv("RIPTRM_TRS_CACHE", raising=False)
        if cg:
            monkeypatch.setenv("RIPTRM_BIG_CG", cg)
        else:
            monkeypatch.delenv("RIPTRM_BIG_CG", raising=False)
        if gb:
            monkeypatch.setenv("RIPTRM_TRS_WS_GB", gb)
        else:
            monkeypatch.delenv("RIPTRM_TRS_WS_GB", raising=False)
        e = _engine(Z)
        r = e.solve(x, y, opt)
        stats[(cg, gb, cache, len(Z))] = e.trs_cache_stats()
        return r

    base = run(Zs, xs, ys)
    hits, total = stats[(None, None, None, B)]
    print(f"eigendecomposition cache: {hits} of {total} subproblems")
    assert total > 0 and 0 < hits <= total, (hits, total)
    for b in range(B):
        lg = base.log(b)
        assert max(lg["iteration"]) == K, (b, max(lg["iteration"]))
        assert all(v is not None for v in lg["mineigvalHw"][1:]), b
    variants = {"grid CG": run(Zs, xs, ys, cg="grid"), "one-workgroup CG": run(Zs, xs, ys, cg="wg"),
                "one slot": run(Zs, xs, ys, gb="0.0004"), "no cache": run(Zs, xs, ys, cache="0")}
    assert stats[(None, None, "0", B)][0] == 0
    for b in (0, 3):
        variants[f"instance {b} alone"] = run(Zs[b:b + 1], xs[b:b + 1], ys[b:b + 1])
    for name, r in variants.items():
        ids = [0] if name == "instance 0 alone" else [3] if name == "instance 3 alone" else range(B)
        for k, b in enumerate(ids):
            ra, rb = r.log(k), base.log(b)
            for key in ("cost", "residual", "normdx", "mineigvalHw"):
                assert ra[key] == rb[key], (name, b, key)
            np.testing.assert_array_equal(r.x[k].cpu().numpy(), base.x[b].cpu().numpy(), err_msg=f"{name} instance {b}")
    ref = O.solve(Zs[0], xs[0], ys[0], _oracle_opt(TRS_solver="Exact_RepMat", second_order_stationarity=True, maxiter=K))
    compare_until_flip(base.log(0), ref.log)


@pytest.mark.timeout(600)
def test_exact_repmat_tri_cg_skip_is_bitwise_neutral(monkeypatch):
    """The tridiagonal path's certified CG skip (csrc/riptrm_tri.h k_tri_solve: from Sturm counts
    either side of 0 and the LDL^T solve T ps = b with its residual, k_cg_wg's bounds show that no CG
    iterate passing RIPTRM.py:246-251 can have p1obj <= xobj, RIPTRM.py:294-298) must not change a
    bit: the bench's own n = 1000 workload (bench.py defaults, instances 0..3 from seed 20251212) with
    the class defaults over K = 5 outer iterations, default vs RIPTRM_CG_SKIP=0 (every CG run to
    SciPy's exit, 10 m iterations where it does not converge): same logs, x and y bit for bit, and
    some CGs really skipped (the test is not vacuous)."""
    import engine
    n, B, K = 1000, 4, 5
    opt = _gpu_opt(TRS_solver="Exact_RepMat", second_order_stationarity=True, maxiter=K)
    runs = {}
    for flag in (None, "0"):
        if flag:
            monkeypatch.setenv("RIPTRM_CG_SKIP", flag)
        else:
            monkeypatch.delenv("RIPTRM_CG_SKIP", raising=False)
        e = engine.NonnegPCABatch(n, B)
        x0, y0 = e.generate_synthetic(20251212, ids=list(range(B)))
        runs[flag] = (e.solve(x0, y0, opt), e.trs_skip_stats())
    (r1, (checked, skipped)), (r0, st0) = runs[None], runs["0"]
    print(f"n = 1000: {checked} subproblems through the skip test, {skipped} CGs skipped")
    assert st0 == (0, 0) and checked > 0 and skipped > 0, (checked, skipped, st0)
    for b in range(B):
        assert max(r1.log(b)["iteration"]) == K
        for key in ("cost", "residual", "normdx", "dxtype", "mineigvalHw", "inner_status", "radius_update"):
            assert r1.log(b)[key] == r0.log(b)[key], (b, key)
    np.testing.assert_array_equal(r1.x.cpu().numpy(), r0.x.cpu().numpy())
    np.testing.assert_array_equal(r1.y.cpu().numpy(), r0.y.cpu().numpy())


@pytest.mark.timeout(900)
def test_exact_repmat_configs1_size_drop_in(monkeypatch):
    """BASELINE configs[1] size (n = 1000) with the reference's class defaults (Exact_RepMat +
    second-order test) through the drop-in: runs (no size cap, RIPTRM.py:324-326), and its first
    outer iteration matches the oracle driven by the eigh formulation of TRSgep (trs_oracle.trs_eigh;
    the pencil's QZ on 1998 x 1998 takes ~90 s per inner step on the CPU, and trs_eigh agrees with it
    to 5e-14 at this size, see tests/test_gpu_trs.py)."""
    from oracle import trs_oracle as TO
    from parity import compare_until_flip
    from problems import NonnegPCAProblem, manviofun
    from RIPTRM import RIPTRM
    Z, x0, y0 = G.generate_instance(1000, 5)
    out = RIPTRM({"maxiter": 1, "tolresid": 0.0, "maxtime": 1e9, "manviofun": manviofun}).run(
        NonnegPCAProblem(Z=Z, initialpoint=x0, initialineqLagmult=y0))
    assert out.name == "RIPTRM_Exact_RepMat" and max(out.log["iteration"]) == 1
    monkeypatch.setattr(TO, "trs_gep", lambda A, a, Del, tol=1e-4: TO.trs_eigh(A, a, Del, tol))
    ref = O.solve(Z, x0, y0, _oracle_opt(maxiter=1, TRS_solver="Exact_RepMat", second_order_stationarity=True))
    compare_until_flip(out.log, ref.log)


@pytest.mark.parametrize("n,B", [(2, 3), (129, 4), (300, 5), (1000, 3), (4000, 9)])
def test_spass_kinds_agree(n, B):
    """The persistent super-tile S-pass (2 x 2 tiles per unit, partials written in bursts) and the
    per-tile S-pass give the same S v to rounding (they add the same products in a different,
    fixed order).  n = 4000, B = 9 is large enough for the automatic choice to pick the super-tile
    kernel (>= 4 units per CU), n = 300 has a partial last super-block, n = 129 a 32-wide edge."""
    Zs, xs, ys, vs = [], [], [], []
    for b in range(B):
        Z, _, _ = G.generate_instance(n, 40 + b)
        x, y = _state(n, 50 + b)
        Zs.append(Z); xs.append(x); ys.append(y)
        vs.append(np.random.RandomState(60 + b).randn(n))
    outs = {}
    for layout in ("sym", "sym2"):
        eng = _engine(np.stack(Zs), layout=layout)
        eng.lib.riptrm_set_spass_kind(eng.ctx.h, 0 if layout == "sym" else 2)
        outs[layout] = eng.hvp(np.stack(xs), np.stack(ys), 0.0123, np.stack(vs)).cpu().numpy()
        if n == 4000:   # automatic choice
            eng.lib.riptrm_set_spass_kind(eng.ctx.h, 1)
            auto = eng.hvp(np.stack(xs), np.stack(ys), 0.0123, np.stack(vs)).cpu().numpy()
            if layout == "sym2":
                np.testing.assert_array_equal(auto, outs["sym2"])
    if n == 4000:
        # default engine (kind 1): a rule on n alone, the super-tile kernel at n = 4000
        eng = _engine(np.stack(Zs))
        cal = eng.spass_calibration()
        assert cal["kernel"] == "k_spass_sup" and cal["ms_per_launch_tile"] == 0.0, cal
        got = eng.hvp(np.stack(xs), np.stack(ys), 0.0123, np.stack(vs)).cpu().numpy()
        np.testing.assert_array_equal(got, outs["sym2"])
        # kind 3: timed at bind, either kernel may win
        import engine
        eng3 = engine.NonnegPCABatch(n, B, layout="sym", spass_kind=3)
        eng3.load_Z(np.stack(Zs))
        cal3 = eng3.spass_calibration()
        assert cal3["ms_per_launch_tile"] > 0 and cal3["ms_per_launch_super"] > 0, cal3
        got3 = eng3.hvp(np.stack(xs), np.stack(ys), 0.0123, np.stack(vs)).cpu().numpy()
        np.testing.assert_array_equal(got3, outs["sym2" if cal3["kernel"] == "k_spass_sup" else "sym"])
    a, b2 = outs["sym"], outs["sym2"]
    scale = np.abs(a).max(axis=1, keepdims=True)
    assert np.max(np.abs(a - b2) / scale) < 1e-13
    if n > 256:   # more than one super-block: a different summation order really ran
        assert not np.array_equal(a, b2)


def test_super_spass_solve_is_deterministic():
    """Two solves with the super-tile S-pass give bitwise identical results (no atomics)."""
    insts = [G.generate_instance(300, 200 + b) for b in range(3)]
    xs = []
    for _ in range(2):
        eng = _engine(np.stack([z for z, _, _ in insts]), layout="sym2")
        res = eng.solve(np.stack([x for _, x, _ in insts]), np.stack([y for _, _, y in insts]), _gpu_opt(maxiter=6))
        xs.append(res.x.cpu().numpy())
    np.testing.assert_array_equal(xs[0], xs[1])


def test_log_longer_than_capacity_is_complete(fixture_n50):
    """A solve whose log outgrows the device capacity (16 records here) is drained to the host
    between lock-step chunks (riptrm_log_rebase): every record arrives, in order, and matches the
    oracle's log row for row."""
    Z, x0, y0 = fixture_n50
    K = 14
    eng = _engine(Z, cap=16)
    res = eng.solve(x0[None], y0[None], _gpu_opt(maxiter=K))
    ref = O.solve(Z, x0, y0, _oracle_opt(maxiter=K))
    gl = res.log(0)
    assert len(gl["iteration"]) == len(ref.log["iteration"]) > 16
    assert int(res.dropped[0]) == 0
    _compare_logs(gl, ref.log)
    full = _engine(Z).solve(x0[None], y0[None], _gpu_opt(maxiter=K))
    notime = lambda a: np.delete(a, 1, axis=1)   # every field but RIPTRM_LOG_TIME
    np.testing.assert_array_equal(notime(res.raw_log[0]), notime(full.raw_log[0]))


def test_log_without_draining_keeps_head_and_latest(fixture_n50):
    """Draining off: the device keeps the first capacity/2 records and a ring of the latest."""
    import engine
    Z, x0, y0 = fixture_n50
    K = 14
    eng = engine.NonnegPCABatch(Z.shape[0], 1, log_capacity=16, drain_logs=False)
    eng.load_Z(Z[None])
    res = eng.solve(x0[None], y0[None], _gpu_opt(maxiter=K))
    full = _engine(Z).solve(x0[None], y0[None], _gpu_opt(maxiter=K))
    a, b = res.raw_log[0], full.raw_log[0]
    assert len(a) == 16 and int(res.dropped[0]) == len(b) - 16
    notime = lambda a: np.delete(a, 1, axis=1)   # every field but RIPTRM_LOG_TIME
    np.testing.assert_array_equal(notime(a[:8]), notime(b[:8]))
    np.testing.assert_array_equal(notime(a[8:]), notime(b[-8:]))
