"""GPU parity of the StableIdentification path (csrc/riptrm_si.hip) against the CPU oracle
(oracle/si_oracle.py, SIVectorized = the kernel's formulas; SIStructured = the reference's
per-constraint wiring) on the reference's fixture dataset/StableIdentification/1 (d = 5, N = 95,
m = 16, 20 initial points).  Manifold formulas are pymanopt restated: parity unpinned at that
boundary; pinned against the published result (analyzer.ipynb: RIPTRM (tCG)
median log10 KKT residual -12.37, Q1 -12.44, Q3 -12.23 within 240 s).

Tolerances: operators 1e-12 relative (fp64, different summation order), teacher-forced tCG same
stop / j and eta within 1e-8, trajectories through tests/parity.py (branch flips at rounding
ties fall back to the outer-level comparison, as for NonnegPCA).
"""
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from conftest import GOLDEN
from oracle import si_oracle as SI

DS = os.path.join(GOLDEN, "si_1")
PTS = "abcdefghijklmnopqrst"


@pytest.fixture(scope="module")
def data():
    return SI.SIData.load(DS)


def _batch(data, B, cap=4096):
    import si
    eng = si.SIBatch(data.d, data.N, data.m, B, log_capacity=cap)
    eng.load(data.X, data.XP, data.h, si.expand_constset(np.loadtxt(os.path.join(DS, "constset.csv"))))
    return eng


def _starts(pts):
    xs, ys = [], []
    for p in pts:
        x0, y0 = SI.load_start(DS, p)
        xs.append(x0)
        ys.append(y0)
    return np.stack(xs), np.stack(ys)


def _gpu_opt(**kw):
    import si
    o = {"TRS_solver": "tCG", "second_order_stationarity": False, "manviofun": si.si_manviofun,
         "tolresid": 0.0, "maxtime": 1e9}
    o.update(kw)
    return o


def _oracle_opt(**kw):
    o = dict(tolresid=0.0, maxtime=1e9, manviofun=SI.si_manvio)
    o.update(kw)
    return o


def test_expand_constset_matches_oracle(data):
    import si
    t = si.expand_constset(np.loadtxt(os.path.join(DS, "constset.csv")))
    assert t.shape == (data.m, 5) == (16, 5)
    for row, (k, r, c, p0, p1) in zip(t, data.cons):
        assert tuple(row) == (k, r, c, p0, p1)


def test_si_hvp_matches_oracle(data):
    B = 8
    xs, ys = _starts(PTS[:B])
    rs = np.random.RandomState(3)
    P = SI.SIVectorized(data)
    vs = np.stack([P.manifold.projection(xs[b], rs.randn(3, 5, 5)) for b in range(B)])
    ys = ys * (0.5 + rs.rand(B, data.m))
    mus = np.array([0.1, 0.05, 1e-3, 1e-6, 0.3, 1e-9, 0.01, 0.2])
    out = _batch(data, B).hvp(xs, ys, mus, vs).cpu().numpy()
    for b in range(B):
        _, _, Hw, _ = P.begin_inner(xs[b], ys[b], mus[b])
        ref = Hw(vs[b])
        err = np.linalg.norm(out[b] - ref) / np.linalg.norm(ref)
        assert err < 1e-12, (b, err)
    # and against the reference-structured wiring
    Ps = SI.SIStructured(data)
    _, _, Hw, _ = Ps.begin_inner(xs[0], ys[0], mus[0])
    ref = Hw(vs[0])
    assert np.linalg.norm(out[0] - ref) / np.linalg.norm(ref) < 1e-12


def test_si_tcg_matches_oracle_teacher_forced(data):
    B = 10
    xs, ys = _starts(PTS[:B])
    rs = np.random.RandomState(5)
    mus = rs.choice([0.1, 0.01, 1e-4], B)
    deltas = rs.choice([np.sqrt(40) / 8, 0.05, 0.2, 1e-3], B)
    eta, _, js, stops = _batch(data, B).tcg(xs, ys, mus, deltas)
    eta = eta.cpu().numpy()
    P = SI.SIVectorized(data)
    from oracle import riptrm_oracle as RO
    for b in range(B):
        _, _, Hw, c = P.begin_inner(xs[b], ys[b], mus[b])
        e, _, j, stop = RO.truncated_conjugate_gradient(P.manifold, Hw, xs[b], c, deltas[b], 1, 0.1, 1, P.manifold.dim)
        assert stops[b] == stop and js[b] == j, (b, stops[b], stop, js[b], j)
        err = np.linalg.norm(eta[b] - e) / max(np.linalg.norm(e), 1e-300)
        assert err <= 1e-8, (b, j, err)


def test_si_solve_start_a_matches_oracle(data):
    from parity import compare_until_flip
    xs, ys = _starts("a")
    eng = _batch(data, 1)
    res = eng.solve(xs, ys, _gpu_opt(maxiter=8))
    ref = SI.solve(data, xs[0], ys[0], _oracle_opt(maxiter=8))
    gl = res.log(0)
    assert abs(gl["residual"][0] - ref.log["residual"][0]) <= 1e-12 * ref.log["residual"][0]
    compare_until_flip(gl, ref.log)
    assert res.stopping_criterion(0).startswith("Max iteration count reached; maxiter=8 after")


def test_si_batch_of_fixture_starts_matches_oracle(data):
    """The problem_initialpoint axis a..t in one launch (shared data, stride 0).  Every start's
    trajectory matches the oracle's up to its first branch flip, which must be a rounding tie of
    the radius-expansion test (or come late), and at the outer level throughout
    (tests/parity.py::compare_until_flip; the two CPU oracles behave the same way,
    tests/test_si_oracle.py)."""
    from parity import compare_until_flip
    xs, ys = _starts(PTS)
    K = 10
    res = _batch(data, len(PTS)).solve(xs, ys, _gpu_opt(maxiter=K))
    for b in range(len(PTS)):
        ref = SI.solve(data, xs[b], ys[b], _oracle_opt(maxiter=K))
        compare_until_flip(res.log(b), ref.log)


def _pins():
    import json
    with open(os.path.join(GOLDEN, "si_1_pins", "oracle_minres.json")) as f:
        return json.load(f)


def _min_log_res(res, B):
    """analyzer.ipynb box-plot cell: per start, log10 of the minimum KKT residual over every log row."""
    out = []
    for b in range(B):
        lg = res.log(b)
        r = np.array(lg["residual"], float)
        out.append((float(np.log10(r.min())), int(lg["iteration"][int(r.argmin())])))
    return out


def test_si_tcg_pinned_to_published_result(data):
    """The reference's own RIPTRM (tCG) result on this fixture (analyzer.ipynb, box-plot cell):
    per-start min log10 KKT residual, start t = -12.475348, quartiles over the 20 starts
    Q1 / median / Q3 = -12.444660 / -12.368153 / -12.225336.  Those minima sit on the rounding
    plateau near mu ~ 1e-13 (outer iteration 33-35), where two fp64 implementations of the same
    algorithm differ by ~0.05 per start: the CPU oracle under the same protocol gives quartiles
    -12.458 / -12.414 / -12.238 (tests/golden/si_1_pins, generated by tests/golden/make_si_pins.py).
    Protocol: maxiter 35, inner_maxiter 300 (the reference ran into its 240 s limit in the stalled
    outer iteration instead).  Bar: quartiles within 0.1 of the published ones, start t within 0.1,
    every start below 1e-11 and its minimum in outer iteration >= 32."""
    pins = _pins()
    pub = pins["published"]
    xs, ys = _starts(PTS)
    opt = pins["protocol"]["tcg"]
    res = _batch(data, len(PTS), cap=16384).solve(xs, ys, _gpu_opt(maxiter=opt["maxiter"], inner_maxiter=opt["inner_maxiter"]))
    got = _min_log_res(res, len(PTS))
    v = np.array([g for g, _ in got])
    q = [np.quantile(v, 0.25), np.median(v), np.quantile(v, 0.75)]
    assert all(abs(a - p) <= 0.1 for a, p in zip(q, pub["tcg_quartiles"])), (q, pub["tcg_quartiles"], pins["tcg_quartiles"])
    assert abs(got[PTS.index("t")][0] - pub["tcg_start_t"]) <= 0.1, got[PTS.index("t")]
    assert (v < -11.0).all() and all(it >= 32 for _, it in got), got


def test_si_exact_pinned_to_published_plateau(data):
    """The reference's RIPTRM (exact) result (analyzer.ipynb, box-plot cell): min log10 KKT residual
    -8.787497 for EVERY one of the 20 starts (Q1 = median = Q3).  The exact runs stall inside outer
    iteration 25 (mu_25 = 4.078e-10: the inner loop keeps taking successful steps at residual
    4 mu_25 = 1.6312e-9 and never meets its tolerance), so the published minimum is a property of the
    algorithm: the mu schedule (RIPTRM.py:866-896), Exact_RepMat's steps (:218-299, :433-444) and the
    second-order test (:599-617) reaching that point from every start.  The CPU oracle reproduces it
    to 1e-9 in log10 (tests/golden/si_1_pins).  The GPU's trajectories leave the reference's at a
    rounding tie of the radius-expansion test |normdx - Delta| <= 1e-15 (RIPTRM.py:672; start a:
    row 4, GPU normdx - Delta = 1.1e-15, CPU 6e-17, scripts/si_exact_log.py), then stall in the
    same outer iteration 25 at the same central-path point but keep taking tiny hard-case steps
    whose residual dips up to ~0.2% below 4 mu_25.  Bar: every start's minimum attained in outer
    iteration 25 and within 2e-3 of -8.787497 in log10 (outer iterations 24 / 26 sit 0.4 away)."""
    pins = _pins()
    opt = pins["protocol"]["exact"]
    xs, ys = _starts(PTS)
    res = _batch(data, len(PTS), cap=8192).solve(xs, ys, _gpu_opt(
        TRS_solver="Exact_RepMat", second_order_stationarity=True, maxiter=opt["maxiter"],
        inner_maxiter=opt["inner_maxiter"]))
    got = _min_log_res(res, len(PTS))
    for p, (g, it) in zip(PTS, got):
        assert abs(g - pins["published"]["exact_every_start"]) <= 2e-3, (p, g, it, got)
        assert it == 25, (p, it, got)


def test_si_per_instance_data_stride(data):
    """Two different problems in one batch (data_stride / cons_stride != 0)."""
    import si
    xs, ys = _starts("ab")
    X2 = data.X * 1.01
    XP2 = data.XP * 0.99
    cons = si.expand_constset(np.loadtxt(os.path.join(DS, "constset.csv")))
    eng = si.SIBatch(data.d, data.N, data.m, 2)
    eng.load(np.stack([data.X, X2]), np.stack([data.XP, XP2]), data.h, np.stack([cons, cons]))
    res = eng.solve(xs, ys, _gpu_opt(maxiter=3))
    d2 = SI.SIData(X2, XP2, data.h, np.loadtxt(os.path.join(DS, "constset.csv")))
    for b, dd in ((0, data), (1, d2)):
        ref = SI.solve(dd, xs[b], ys[b], _oracle_opt(maxiter=3))
        assert abs(res.log(b)["residual"][0] - ref.log["residual"][0]) <= 1e-12 * ref.log["residual"][0]
        assert abs(res.log(b)["cost"][0] - ref.log["cost"][0]) <= 1e-12 * abs(ref.log["cost"][0])


def test_si_drop_in_run_and_simulator(tmp_path):
    """RIPTRM(option).run(SIProblem) from the reference dataset layout, CSVs via save_output."""
    import shutil
    import pandas as pd
    from simulator import save_output
    from si import SICoordinator
    from RIPTRM import RIPTRM
    d = tmp_path / "dataset" / "StableIdentification" / "1"
    d.mkdir(parents=True)
    for f in os.listdir(DS):
        shutil.copy(os.path.join(DS, f), d / f)
    cfg = {"problem_name": "StableIdentification", "problem_instance": 1, "problem_initialpoint": "c",
           "is_X_noisy": True, "Xset": [1, 2, 3, 4, 5], "h": 0.02}
    prob = SICoordinator(cfg, root=str(tmp_path)).run()
    out = RIPTRM(_gpu_opt(maxiter=4)).run(prob)
    assert out.name == "RIPTRM_tCG" and len(out.x) == 3 and out.ineqLagmult.shape == (16,)
    save_output(str(tmp_path / "out"), out.name, out)
    lg = pd.read_csv(tmp_path / "out" / "RIPTRM_tCG_log.csv")
    assert lg["iteration"].max() == 4
    x0, y0 = SI.load_start(DS, "c")
    ref = SI.solve(SI.SIData.load(DS), x0, y0, _oracle_opt(maxiter=4))
    assert abs(lg["residual"][0] - ref.log["residual"][0]) <= 1e-12 * ref.log["residual"][0]


def test_si_deterministic(data):
    xs, ys = _starts("abcd")
    a = _batch(data, 4).solve(xs, ys, _gpu_opt(maxiter=5))
    b = _batch(data, 4).solve(xs[::-1].copy(), ys[::-1].copy(), _gpu_opt(maxiter=5))
    np.testing.assert_array_equal(a.x.cpu().numpy(), b.x.cpu().numpy()[::-1])


@pytest.mark.parametrize("sos", [True, False])
def test_si_exact_repmat_matches_oracle(data, sos):
    """TRS_solver = 'Exact_RepMat' (RIPTRM.py:433-444): the matrix of HwCur in a tangent basis (40 HVPs
    in-kernel), TRSgep on the device (csrc/riptrm_trs.h), and with second_order_stationarity the
    smallest eigenvalue of HwNew's matrix at every trial point (RIPTRM.py:599-617) against the oracle
    (trs_oracle: the reference's 2n x 2n pencil).  Same bar as the tCG trajectories."""
    from parity import compare_until_flip
    xs, ys = _starts("abc")
    K = 4
    opt = dict(TRS_solver="Exact_RepMat", second_order_stationarity=sos, maxiter=K)
    res = _batch(data, 3).solve(xs, ys, _gpu_opt(**opt))
    for b in range(3):
        ref = SI.solve(data, xs[b], ys[b], _oracle_opt(**opt))
        gl = res.log(b)
        kinds = [k for k in gl["dxtype"] if k is not None]
        assert kinds and all(k in ("boundary", "interior", "hardcase_1") for k in kinds), kinds
        mins = [v for v in gl["mineigvalHw"] if v is not None]
        assert (len(mins) > 0) == sos
        compare_until_flip(gl, ref.log)


def test_si_reference_default_options_use_exact_repmat(tmp_path):
    """RIPTRM's class defaults (RIPTRM.py:325-326): Exact_RepMat with the second-order test."""
    from si import SICoordinator
    from RIPTRM import RIPTRM
    import shutil
    d = tmp_path / "dataset" / "StableIdentification" / "1"
    d.mkdir(parents=True)
    for f in os.listdir(DS):
        shutil.copy(os.path.join(DS, f), d / f)
    cfg = {"problem_name": "StableIdentification", "problem_instance": 1, "problem_initialpoint": "a",
           "is_X_noisy": True, "Xset": [1, 2, 3, 4, 5], "h": 0.02}
    prob = SICoordinator(cfg, root=str(tmp_path)).run()
    import si
    out = RIPTRM({"maxiter": 2, "tolresid": 0.0, "maxtime": 1e9, "manviofun": si.si_manviofun}).run(prob)
    assert out.name == "RIPTRM_Exact_RepMat"
    assert any(v is not None for v in out.log["mineigvalHw"])
