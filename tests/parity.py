"""Trajectory comparator shared by the GPU parity tests and the CPU calibration test.

Two fp64 implementations of RIPTRM that differ only in summation order (the GPU's tree
reductions vs BLAS, or the reference-structured vs the vectorised CPU oracle) take the SAME
branch decisions on these inputs but their iterates drift at the level of CG's rounding
sensitivity.  Calibration on the CPU (tests/test_oracle.py::test_comparator_calibration):
outer-iterate rows agree to ~1e-7 relative in the KKT residual, while the KKT gradient norm at
a converged row (a ~1e-8 residual of the inner solve) and intermediate trial rows (points
produced by a MAX_INNER_ITER tCG) differ by up to O(1) relative.
The bar therefore is:
* identical branch decisions: iteration, num_inner, inner_status, dxtype, radius_update,
  dual_clipping (and so identical row counts);
* outer-iterate rows (inner_status None/'converged'): |g-r| <= 1e-4 |r| + 1e-5 max|r| for the
  quantities of the iterate (residual, cost, violations, mu, TR radius, max |y|);
* the quantities of the tCG step / trial point (normdx, minxfeasi, minyfeasi, compl, ared/pred)
  and every value on a trial row:
  |g-r| <= |r| or |g-r| <= 1e-2 max|r| (observed between the CPU oracles: step norms 54% apart
  after a MAX_INNER_ITER tCG with identical branches, n=200 seed 101, row 45);
* plus an absolute 1e-14 everywhere (e.g. ||x|| - 1 is pure rounding, ~1e-16).

That calibrated trial bound is loose by design.  The NonnegPCA GPU solve tests tighten it with
an ENVELOPE: five CPU oracle runs that are the same arithmetic in another summation order
(order_variants: dgemv, and dsymv on four symmetric permutations) measure how far this very
trajectory moves under rounding, column by column; the GPU's trial values must stay within 10x
that (compare_logs(envelope=...)), its tCG exit indices within the variants' spread
(compare_tcg_iters), and only a budgeted few instances per test (excursion_budget) may show a
rare amplification past it -- still inside the calibrated bound, as a further CPU variant does in
~1 comparison of 40.
"""
import numpy as np


class BranchFlip(AssertionError):
    """The two trajectories took a different branch at some inner iteration."""


BRANCH_KEYS = ("iteration", "num_inner", "inner_status", "dxtype", "radius_update", "dual_clipping")
VALUE_KEYS = ("residual", "cost", "gradnorm", "complviolation", "dualviolation", "manviolation",
              "maxviolation", "meanviolation", "mu", "normdx", "TR_radius", "minxfeasi", "minyfeasi",
              "compl", "ared/pred", "maxabsLagmult", "mineigvalHw")
# properties of the tCG step / trial point rather than of the iterate: trial bounds on every row
STEP_KEYS = ("normdx", "minxfeasi", "minyfeasi", "compl", "ared/pred", "mineigvalHw")


def _col(log, k):
    return np.array([np.nan if v is None else float(v) for v in log[k]], dtype=float)


def compare_logs(gl, rl, rtol=1e-4, ascale=1e-5, trial_rtol=1.0, trial_ascale=1e-2, atol=1e-14,
                 envelope=None, env_mult=10.0, env_rel=1e-9, excursions=None):
    """envelope (see `envelope`): per key and row, the distance between the reference log and
    order-perturbed oracle runs that share its branches up to that row.  Where it is given, the
    trial-bar rows of a column must satisfy |g - r| <= (env_mult * E + env_rel) |r| + atol with E
    the variants' largest relative deviation over the column's trial-bar rows, instead of the
    calibrated trial_rtol / trial_ascale bound (rows no variant covers, past every variant's own
    first flip, keep that bound).  Column- rather than row-level, and 10x rather than 3x: a
    further CPU order variant exceeds the row-level 3x envelope of three variants by up to 470x
    and the column-level one by up to 8.2x.  Even so, with five variants about one comparison in
    forty shows a rare amplification (a trial value 1000x past every variant, still inside the
    calibrated bound; tests/test_oracle.py::test_envelope_calibration).  Pass a list as
    `excursions` to collect such columns instead of failing; the caller then bounds how many
    instances of a test may have one (excursion_budget)."""
    assert list(gl.keys()) == list(rl.keys()), (list(gl.keys()), list(rl.keys()))
    for k in BRANCH_KEYS:
        if k in gl and gl[k] != rl[k]:
            m = min(len(gl[k]), len(rl[k]))
            first = next((i for i in range(m) if gl[k][i] != rl[k][i]), m)
            raise BranchFlip(f"{k} differs first at row {first}")
    outer = np.array([s in (None, "converged") for s in rl["inner_status"]])
    for k in VALUE_KEYS:
        if k not in gl:
            continue
        g, r = _col(gl, k), _col(rl, k)
        assert np.array_equal(np.isnan(g), np.isnan(r)), k
        m = ~np.isnan(r)
        if not m.any():
            continue
        scale = np.max(np.abs(r[m])) or 1.0
        d = np.abs(g - r)
        ok_outer = d <= rtol * np.abs(r) + ascale * scale + atol
        ok_trial = (d <= trial_rtol * np.abs(r)) | (d <= trial_ascale * scale + atol)
        if envelope is not None and k in envelope:
            # outer rows: past rtol only where the variants themselves move that row (row-level,
            # absolute: |g - r| <= env_mult x max_v |v - r| at the row; late in a K = 20 window the
            # radius carried out of an outer iteration inherits the erratic tCG exit's normdx)
            er = envelope[k][:len(r)]
            ok_outer = ok_outer | (~np.isnan(er) & (d <= env_mult * np.where(np.isnan(er), 0.0, er) + atol))
            # column-level envelope: over the rows the variants cover, the largest relative
            # deviation of this column stays within env_mult x the variants' largest one
            e = envelope[k][:len(r)]
            den = np.maximum(np.abs(r), 1e-12 * scale)
            cov = m & ~np.isnan(e) & ~(outer if k not in STEP_KEYS else np.zeros_like(outer))
            if cov.any():
                lim = env_mult * np.max(e[cov] / den[cov]) + env_rel
                ok_env = d <= lim * den + atol
                rows_t = m & ~(outer if k not in STEP_KEYS else np.zeros_like(outer))
                over = rows_t & ~np.isnan(e) & ~ok_env
                if over.any() and excursions is not None and not (over & ~ok_trial).any():
                    # within the calibrated bound but past the envelope: a rare amplification
                    # (the caller budgets these across a test's instances)
                    excursions.append((k, [int(i) for i in np.nonzero(over)[0][:5]]))
                else:
                    ok_trial = np.where(np.isnan(e), ok_trial, ok_env)
        rows_outer = outer if k not in STEP_KEYS else np.zeros_like(outer)
        bad = m & np.where(rows_outer, ~ok_outer, ~ok_trial)
        assert not bad.any(), (k, np.nonzero(bad)[0][:5], g[bad][:5], r[bad][:5],
                               "envelope", None if envelope is None or k not in envelope else envelope[k][:len(r)][bad][:5],
                               "variant flips", None if envelope is None else envelope.get("_flips"))


def outer_rows(log):
    """Row index of each outer iterate: row 0 and the last row of every outer iteration."""
    it = log["iteration"]
    rows = [0]
    for r in range(1, len(it)):
        if r == len(it) - 1 or it[r + 1] != it[r]:
            rows.append(r)
    return rows


def compare_outer(gl, rl, rtol=1e-3, tol_mult=10.0):
    """Outer-level agreement for trajectories whose inner branches differ (a rounding tie, as
    the CPU oracles themselves show on some instances): same outer iterations, same end state of
    each, and the KKT residual of every outer iterate within rtol or within tol_mult times the
    inner stopping tolerance max(mu, 1e-14) of that outer iteration (RIPTRM.py:320)."""
    go, ro = outer_rows(gl), outer_rows(rl)
    assert [gl["iteration"][i] for i in go] == [rl["iteration"][i] for i in ro]
    assert [gl["inner_status"][i] for i in go] == [rl["inner_status"][i] for i in ro]
    for a, b in zip(go, ro):
        g, r = float(gl["residual"][a]), float(rl["residual"][b])
        tol = tol_mult * max(float(rl["mu"][b]), 1e-14)
        assert abs(g - r) <= max(rtol * abs(r), tol), (rl["iteration"][b], g, r)


def first_branch_flip(gl, rl):
    """(row, key) of the first row whose branch decisions differ, or None."""
    first = None
    for k in BRANCH_KEYS:
        if k not in gl:
            continue
        m = min(len(gl[k]), len(rl[k]))
        f = next((i for i in range(m) if gl[k][i] != rl[k][i]), None)
        if f is None and len(gl[k]) != len(rl[k]):
            f = m
        if f is not None and (first is None or f < first[0]):
            first = (f, k)
    return first


def _prefix(log, n):
    return {k: v[:n] for k, v in log.items()}


def is_radius_tie(gl, rl, row, rel=1e-12):
    """RIPTRM.py:672 expands the radius only if |normdx - Delta| <= 1e-15: for a boundary step
    normdx equals Delta up to the rounding of the metric norm (1e-15..1e-14 relative on the SPD
    factors), so 'expanded' vs 'unchanged' is a coin flip between two fp64 implementations."""
    if {gl["radius_update"][row], rl["radius_update"][row]} != {"expanded", "unchanged"}:
        return False
    for lg in (gl, rl):
        nd, tr = float(lg["normdx"][row]), float(lg["TR_radius"][row])
        if abs(nd - tr) > rel * tr:
            return False
    return True


def compare_until_flip(gl, rl, tight_rows=20, late_row=20):
    """Trajectory comparison for problems whose iterates are sensitive to rounding
    (StableIdentification: the two CPU oracles, identical up to summation order, keep identical
    branches for tens of rows but drift apart by O(1) in the residual after 25-45 rows, and their
    first branch flip is usually a radius-expansion tie; tests/test_si_oracle.py): the first
    min(first flip, tight_rows) rows meet compare_logs' bar; the first flip is a radius-update tie
    (is_radius_tie) or comes after `late_row` rows; the outer iterates agree at the level of the
    inner tolerance (compare_outer).  Returns the flip (row, key) or None."""
    flip = first_branch_flip(gl, rl)
    n = tight_rows if flip is None else min(flip[0], tight_rows)
    if n > 0:
        compare_logs(_prefix(gl, n), _prefix(rl, n))
    if flip is not None:
        row, key = flip
        assert (key == "radius_update" and is_radius_tie(gl, rl, row)) or row >= late_row, \
            (flip, gl[key][row], rl[key][row], gl["normdx"][row], rl["normdx"][row], gl["TR_radius"][row])
    compare_outer(gl, rl)
    return flip


# ---- envelopes of order-perturbed oracle runs -------------------------------------------------

def order_variants(Z, x0, y0, option, S=None, seeds=(1, 2, 6, 7), structured_too=False):
    """Oracle runs that are the same arithmetic in another summation order: dgemv instead of
    dsymv, and dsymv on symmetric permutations P S P^T (x0, y0 permuted; every logged quantity is
    permutation invariant).  The spread of these runs around the reference run is the rounding
    sensitivity of the trajectory itself (the method of test_gpu_n4000's teacher-forced test)."""
    from oracle import riptrm_oracle as O
    S = np.asarray(Z, dtype=np.float64) + np.asarray(Z, dtype=np.float64).T if S is None else S
    out = [O.RIPTRMOracle(option).run(O.NonnegPCAVectorized(S, S=S, symv=False), x0, y0)]
    for sd in seeds:
        # progress on stdout: long runs (n = 4000) must not look hung to the GPU job runner
        print(f"[parity] order variant {len(out)}/{len(seeds) + 1} done (n = {S.shape[0]})", flush=True)
        p = np.random.RandomState(sd).permutation(S.shape[0])
        Sp = np.ascontiguousarray(S[p][:, p])
        out.append(O.RIPTRMOracle(option).run(O.NonnegPCAVectorized(Sp, S=Sp), x0[p], y0[p]))
    if structured_too:
        out.append(O.RIPTRMOracle(option).run(O.NonnegPCAStructured(Z), x0, y0))
    return out


def envelope(ref, variants):
    """Per VALUE_KEYS column: row-wise max |v - r| over the variants whose branch decisions agree
    with the reference up to that row (NaN where none does).  Key "_tcg": per inner step, the
    largest |j_v - j_r| of the tCG exit iteration over the same variants."""
    rl = ref.log
    nrows = len(rl["iteration"])
    env = {}
    flips = [first_branch_flip(v.log, rl) for v in variants]
    for k in VALUE_KEYS:
        if k not in rl:
            continue
        r = _col(rl, k)
        e = np.full(nrows, np.nan)
        for v, f in zip(variants, flips):
            lim = nrows if f is None else f[0]
            d = np.abs(_col(v.log, k)[:lim] - r[:lim])
            d = np.where(np.isnan(d), 0.0, d)
            e[:lim] = np.fmax(e[:lim], d)
        env[k] = e
    steps = len(ref.trace)
    dj = np.full(steps, np.nan)
    for v, f in zip(variants, flips):
        lim = min(steps, len(v.trace), steps if f is None else max(0, f[0] - 1))
        a = np.array([t["tcg_iters"] for t in v.trace[:lim]], float)
        b = np.array([t["tcg_iters"] for t in ref.trace[:lim]], float)
        dj[:lim] = np.fmax(dj[:lim], np.abs(a - b))
    env["_tcg"] = dj
    env["_flips"] = flips
    return env


def excursion_budget(instances: int) -> int:
    """Instances of one test allowed an envelope excursion: the CPU calibration rate is ~1/40
    per comparison; allow 10% of the instances (at least one)."""
    return max(1, instances // 10)


def tcg_exit_reachable(P, state, target, drift, trials=6, seed=0, slack=2, rel=0.005):
    """A tCG exit index that differs from the oracle's by more than its order variants' spread is
    still a rounding quantity if the oracle's own tCG (RIPTRM.py:41-216), started from the oracle's
    state at that inner step perturbed at sizes from 1e-14 up to the drift the trajectories had
    accumulated (prefix_deviation, capped at 1e-8), exits at indices whose range covers the GPU's
    (within max(slack, rel j)).  Long CG runs at mu ~ 1e-7 (hundreds of iterations, condition numbers
    ~ 1/mu) cross the residual target on a plateau, where such perturbations move the exit a lot.
    state = (x, y, mu, Delta, inner_iteration, inner_option) as StateRecorder keeps it.  Returns the
    (min, max) exit indices seen when the target is covered, else None."""
    from oracle import riptrm_oracle as O
    x, y, mu, Delta = state[:4]
    n = x.shape[0]
    rs = np.random.RandomState(seed)
    sizes = np.logspace(-14, np.log10(max(drift, 1e-14)), max(1, int(np.ceil(np.log10(max(drift, 1e-14)) + 14)) + 1))
    lo, hi = None, None
    tol = max(slack, rel * target)
    for t in range(trials * len(sizes)):
        eps = sizes[t // trials] * (0.5 + rs.rand())
        xp = x * (1.0 + eps * rs.randn(n))
        xp = xp / np.linalg.norm(xp)
        yp = y * (1.0 + eps * rs.randn(n))
        _, _, Hw, c = P.begin_inner(xp, yp, mu)
        _, _, j, _ = O.truncated_conjugate_gradient(P.manifold, Hw, xp, c, Delta, 1, 0.1, 1, n - 1)
        lo = j if lo is None else min(lo, j)
        hi = j if hi is None else max(hi, j)
        if lo - tol <= target <= hi + tol:
            return (lo, hi)
    return None


def compare_tcg_iters(g_iters, ref, env, mult=3.0, rel=0.005, slack=2, reachable=None):
    """tCG exit iterations per inner step (GPU log rows 1.. = oracle trace) and their total: each
    within max(slack, mult x the variants' largest |dj| over the run, rel x j), the total within
    max(mult x the variants' largest per-step |dj| x steps moved, rel x total).  CG's exit index
    is itself a rounding quantity near a stopping threshold (a fourth CPU order variant moves
    short runs by one or two iterations where the three variants agree)."""
    r = np.array([t["tcg_iters"] for t in ref.trace], float)
    g = np.asarray(g_iters, float)[:len(r)]
    assert len(g) == len(r), (len(g), len(r))
    dj = env["_tcg"][:len(r)]
    djmax = float(np.nanmax(dj)) if np.any(~np.isnan(dj)) else 0.0
    lim = np.maximum(np.maximum(slack, mult * djmax), rel * r)
    bad = np.abs(g - r) > lim
    if bad.any() and reachable is not None:
        # reachable(i, j_gpu): the exit index of inner step i is a rounding quantity there
        # (tcg_exit_reachable); at most 8 such steps per instance are examined
        idx = np.nonzero(bad)[0]
        assert len(idx) <= 8, (idx[:10], g[bad][:10], r[bad][:10], djmax)
        for i in idx:
            assert reachable(int(i), int(g[i])) is not None, (int(i), g[i], r[i], djmax)
        keep = ~bad
        g, r = g[keep], r[keep]
        bad = np.zeros(len(g), bool)
    assert not bad.any(), (np.nonzero(bad)[0][:5], g[bad][:5], r[bad][:5], djmax)
    moved = int(np.sum(g != r))
    assert abs(g.sum() - r.sum()) <= max(slack * moved, mult * djmax * moved, rel * r.sum()), (g.sum(), r.sum())


# ---- classified branch flips ------------------------------------------------------------------

def column_deviation(a, r, k):
    """max over rows of |a - r| / max(|r|, 1e-12 max|r|) for column k (rows both logs have)."""
    m = min(len(a[k]), len(r[k]))
    g, v = _col(a, k)[:m], _col(r, k)[:m]
    ok = ~np.isnan(g) & ~np.isnan(v)
    if not ok.any():
        return 0.0
    scale = np.max(np.abs(v[ok])) or 1.0
    return float(np.max(np.abs(g[ok] - v[ok]) / np.maximum(np.abs(v[ok]), 1e-12 * scale)))


DRIFT_CAP = 1e-8


def prefix_deviation(gl, rl, rows, cap=DRIFT_CAP):
    """Relative deviation of the iterate quantities (cost, residual, max |y|) on the OUTER-iterate
    rows (row 0 and each outer iteration's last row) among the first `rows` rows: the drift the
    two trajectories have accumulated before a flip.  Trial rows are left out (their values differ
    by up to O(1) between any two fp64 implementations), and the result is capped at `cap`."""
    keep = [i for i in outer_rows(rl) if i < rows and i < len(gl["iteration"])]
    if not keep:
        return 0.0
    p = {k: [v[i] for i in keep] for k, v in gl.items()}
    q = {k: [v[i] for i in keep] for k, v in rl.items()}
    return min(cap, max(column_deviation(p, q, k) for k in ("cost", "residual", "maxabsLagmult")))


def sphere_perturb(x, y, eps, rs):
    """relative perturbation of a Sphere point (renormalised) and of the multipliers"""
    xp = x * (1.0 + eps * rs.randn(x.shape[0]))
    return xp / np.linalg.norm(xp), y * (1.0 + eps * rs.randn(y.shape[0]))


def si_perturb(x, y, eps, rs):
    """relative perturbation of a Product(Skew, SPD, SPD) point that keeps its structure (J skew,
    R and Q symmetric: an elementwise factor 1 + eps sym(noise)) and of the multipliers"""
    xp = np.empty_like(x)
    a = rs.randn(*x.shape[1:])
    xp[0] = x[0] * (1.0 + eps * (a + a.T) / 2)
    for k in (1, 2):
        b = rs.randn(*x.shape[1:])
        xp[k] = x[k] * (1.0 + eps * (b + b.T) / 2)
    return xp, y * (1.0 + eps * rs.randn(y.shape[0]))


def classify_flip(step, P, states, gl, rl, flip, trials=8, seed=0, perturb=sphere_perturb, drift=None):
    """A branch flip at log row `flip[0]` (key flip[1]) is a rounding-driven one if the GPU's decision
    is reachable from the ORACLE's own state at that inner step perturbed at any size from 1e-14 up
    to the drift the two trajectories had accumulated before it on their outer iterates
    (prefix_deviation, capped at DRIFT_CAP = 1e-8 relative): random relative
    perturbations of x (kept on the sphere) and y, `trials` per decade, each run through the
    oracle's inner_step `step` (RIPTRM.py:707-783).  Decisions that flip this way are
    either ties (|normdx - Delta| <= 1e-15, RIPTRM.py:672) or the erratic tail of an ill-conditioned
    tCG (residual ratios jumping 10x between iterations near the exit): the two CPU oracles flip
    there too (tests/test_oracle.py).  A decision with a real margin is not reproduced (the negative
    control there).  states[r - 1] = (x, y, mu, Delta, inner_iteration, inner_option) of the inner
    step that wrote row r.  Returns the perturbation size that reproduced it, or None."""
    row, key = flip
    if row < 1 or row - 1 >= len(states):
        return None
    x, y, mu, Delta, it, iopt = states[row - 1]
    drift = max(prefix_deviation(gl, rl, row) if drift is None else min(drift, DRIFT_CAP), 1e-14)
    want = gl[key][row]
    rs = np.random.RandomState(seed)
    sizes = np.logspace(-14, np.log10(drift), max(1, int(np.ceil(np.log10(drift) + 14)) + 1))
    for t in range(trials * len(sizes)):
        eps = sizes[t // trials] * (0.5 + rs.rand())
        xp, yp = perturb(x, y, eps, rs)
        _, _, _, _, info = step(P, xp, yp, mu, Delta, it, iopt)
        if info.get(key) == want:
            return eps
    return None


class StateRecorder:
    """Wraps an oracle so its inner steps record their starting state (for classify_flip)."""

    def __init__(self, oracle):
        self.oracle = oracle
        self.states = []
        inner = oracle.inner_step
        self.step = inner   # the unwrapped inner step (classify_flip's probe)

        def rec(P, x, y, mu, Delta, inner_iteration, inner_option):
            self.states.append((x.copy(), y.copy(), mu, Delta, inner_iteration, dict(inner_option)))
            return inner(P, x, y, mu, Delta, inner_iteration, inner_option)

        oracle.inner_step = rec


# ---- one GPU instance against the oracle ----------------------------------------------------

def variant_supports_flip(variants, gl, rl, flip):
    """A branch flip of the GPU log at row r is rounding-driven also if the oracle's own order
    variants (the same arithmetic in another summation order: order_variants) leave the reference
    run's branches there: one of them takes the GPU's decision at row r, or one of them already
    flips at a row <= r (past that row the reference trajectory is not stable under reordering, so
    its branch decisions are no target; the outer iterates must still agree, compare_outer).
    Late in a K = 20 window (mu ~ 1e-8) the acceptance test ared > 0.1 pred (RIPTRM.py:677) compares
    merit differences of ~1e-15 |phi|, and the four dsymv permutations split there themselves."""
    row, key = flip
    for v in variants:
        vf = first_branch_flip(v.log, rl)
        if vf is None:
            continue
        if vf[0] < row:
            return True
        if vf[0] == row and row < len(v.log[key]) and v.log[key][row] == gl[key][row]:
            return True
    return False


def variant_decorrelated(ra, variants, flip, rel=1e-3):
    """The oracle's own order variants, with the reference's branches, already carry a trust-region
    radius more than `rel` (relative) away from the reference's on some row before the flip: the
    state the later decisions act on has decorrelated under summation order alone (late in a K = 20
    window an ill-conditioned tCG exit -- normdx 5% apart from states equal to 1e-15 -- sets the
    radius through gamma normdx after a primal-infeasible trial, RIPTRM.py:687), so the reference's
    branches past that row are no target for any fp64 implementation.  Such a flip always counts
    against the budget, and the outer iterates must still agree (compare_outer)."""
    row = flip[0]
    env = envelope(ra, variants)
    e = env.get("TR_radius")
    if e is None:
        return False
    r = np.abs(_col(ra.log, "TR_radius"))
    lim = min(row, len(e), len(r))
    if lim < 1:
        return False
    d = e[:lim] / np.maximum(r[:lim], 1e-300)
    d = d[~np.isnan(d)]
    return bool(d.size and d.max() > rel)


EPS = 2.220446049250313e-16


def decision_margins(step, P, state):
    """The oracle's acceptance / radius decision at one inner step (RIPTRM.py:640-683), with the
    forward error of its inputs: ared = phi(x) - phi(x+) (+ reg) and pred = -<Hw dx, dx>/2 - <c, dx>
    (+ reg), phi(x) = f(x) - mu sum log s(x) (RIPTRM.py:644-660).  phi(x) and phi(x+) are each
    evaluated with an independent rounding error (the GPU's f = -x^T (S x) / 2 with tree sums, the
    oracle's BLAS), bounded by eps sqrt(n) (sum_ij |x_i| |S_ij| |x_j| / 2 + mu sum |log s_i|) per
    point (random-walk growth of n-term sums); pred's by eps sqrt(n) (sum |(Hw dx)_i dx_i| / 2 +
    sum |c_i dx_i|).  Input perturbations move phi(x) and phi(x+) together and cannot show this
    evaluation noise, which is what decides ared > rho pred once ared and pred are ~ reg.
    state = StateRecorder's (x, y, mu, Delta, inner_iteration, inner_option).  Returns a dict
    (ared, pred, err_ared, err_pred) or None when the step did not reach the ratio test."""
    orc = getattr(step, "__self__", None)
    if orc is None:
        return None
    x, y, mu, Delta, it, iopt = state
    got = {}
    orig = orc.update_xy_TR_radius

    def wrap(P_, x_, y_, sCur, Hw, c, dx, normdx, xNew, yNew, sNew, mu_, Delta_):
        out = orig(P_, x_, y_, sCur, Hw, c, dx, normdx, xNew, yNew, sNew, mu_, Delta_)
        n = x_.size
        S = getattr(P_, "S", None)

        def f_scale(xx):
            if S is not None:
                ax = np.abs(xx).ravel()
                return 0.5 * float(ax @ (np.abs(S) @ ax))
            return abs(P_.cost(xx))

        lb0 = P_.cost(x_) - mu_ * np.sum(np.log(sCur))
        lb1 = P_.cost(xNew) - mu_ * np.sum(np.log(sNew))
        reg = max(1, abs(lb0)) * EPS * orc.option['reduction_regularization']
        hd = Hw(dx)
        M = P_.manifold
        pred = 0 - 0.5 * M.inner_product(x_, hd, dx) - M.inner_product(x_, c, dx)
        rn = np.sqrt(n)
        got.update(ared=(lb0 - lb1) + reg, pred=pred + reg,
                   err_ared=EPS * rn * (f_scale(x_) + f_scale(xNew)
                                        + mu_ * (np.sum(np.abs(np.log(sCur))) + np.sum(np.abs(np.log(sNew))))),
                   err_pred=EPS * rn * (0.5 * float(np.sum(np.abs(hd * dx))) + float(np.sum(np.abs(c * dx)))))
        return out

    orc.update_xy_TR_radius = wrap
    try:
        step(P, x, y, mu, Delta, it, iopt)
    finally:
        del orc.update_xy_TR_radius
    return got or None


def decision_tie(step, P, states, gl, rl, flip):
    """A flipped acceptance (inner_status successful / unsuccessful: ared > rho pred, rho = 0.1) or
    radius decision (reduced / unchanged: ared < pred / 4) whose margin at the oracle's own state
    lies within the forward error of ared and pred (decision_margins) is a rounding tie.  Returns
    the margin / error ratio, or None."""
    row, key = flip
    pair = {gl[key][row], rl[key][row]}
    if key == "inner_status" and pair == {"successful", "unsuccessful"}:
        t = 0.1
    elif key == "radius_update" and pair == {"reduced", "unchanged"}:
        t = 0.25
    else:
        return None
    if row < 1 or row - 1 >= len(states):
        return None
    m = decision_margins(step, P, states[row - 1])
    if not m:
        return None
    margin = abs(m["ared"] - t * m["pred"])
    err = m["err_ared"] + t * m["err_pred"]
    return margin / err if margin <= err else None


def forced_outer_flip(gl, flip, P, opt, resume):
    """Teacher forcing at the outer boundary, for a flip the classifiers above cannot reproduce from
    the ORACLE's state because the two trajectories have drifted apart over many outer iterations
    (within the order variants' envelope, but past DRIFT_CAP): the GPU's own iterate at the head of
    the flip's outer iteration k (`resume(k - 1)` -> x, y, mu, Delta of the device solve paused
    there) goes into the oracle's inner_run for outer iteration k (RIPTRM.py:785-847).  From the
    same state, the oracle must take the GPU's branches on every row of iteration k through the
    flip row, with values within the calibrated bar (compare_logs) -- i.e. the GPU's decision is
    the reference's decision at the GPU's own state -- or its own first flip against the GPU there
    must be a classified rounding tie (classify_flip with the drift of iteration k's earlier rows,
    decision_tie, is_radius_tie).  Returns (k, row, eps) or None."""
    from oracle import riptrm_oracle as O
    row = flip[0]
    k = int(gl["iteration"][row])
    rows_k = [i for i in range(1, len(gl["iteration"])) if gl["iteration"][i] == k]
    if k < 1 or not rows_k or rows_k != list(range(rows_k[0], rows_k[-1] + 1)):
        return None
    h = rows_k[0] - 1
    x, y, mu_dev, delta = resume(k - 1)
    orc = O.RIPTRMOracle(opt)
    rec = StateRecorder(orc)
    o = orc.option
    mu = O.mu_schedule(opt, k)[k - 1]
    assert abs(mu - mu_dev) <= 1e-14 * mu, (mu, mu_dev)
    Delta = max(float(delta), o['minimal_initial_TR_radius'])
    inner_option = {"stopping_criterion_Lagrangian": o['forcing_function_Lagrangian'](mu),
                    "stopping_criterion_complementarity": o['forcing_function_complementarity'](mu)}
    x = np.asarray(x, np.float64)
    y = np.asarray(y, np.float64)
    t0 = orc.clock()
    orc.add_log(0, t0, orc.evaluation(P, x, x, y), orc.solver_status(y, mu, True, None))   # a head row (dropped)
    orc.inner_run(P, k, t0, x, y, mu, Delta, inner_option)
    # the GPU's own rows 0..h in front of both (identical: the columns keep their scale, and the
    # continuation's row i is global row h + i)
    keys = [key for key in orc.log if key in gl]
    sub_g = {key: list(gl[key][:h + 1]) + [gl[key][i] for i in rows_k] for key in keys}
    sub_o = {key: list(gl[key][:h + 1]) + list(orc.log[key][1:]) for key in keys}
    states = [None] * h + rec.states
    f = first_branch_flip(sub_g, sub_o)
    if f is None or f[0] > row:
        compare_logs(_prefix(sub_g, row + 1), _prefix(sub_o, row + 1))
        return (k, row, 0.0)
    if f[0] > h + 1:
        compare_logs(_prefix(sub_g, f[0]), _prefix(sub_o, f[0]))
    pre = lambda lg: {key: v[h + 1:f[0]] for key, v in lg.items()}   # noqa: E731
    drift = max([column_deviation(pre(sub_g), pre(sub_o), key) for key in ("cost", "residual")] + [0.0])
    eps = classify_flip(rec.step, P, states, sub_g, sub_o, f, drift=drift)
    if eps is None and decision_tie(rec.step, P, states, sub_g, sub_o, f) is not None:
        eps = 0.0
    if eps is None and f[1] == "radius_update" and is_radius_tie(sub_g, sub_o, f[0]):
        eps = 0.0
    return None if eps is None else (k, f[0], eps)


def check_against(gl, ra, states, variants, P, step, gpu_x=None, gpu_tcg=None, resume=None, opt=None):
    """check_instance's bar, given the oracle's reference run `ra` (its inner steps' starting
    states recorded: StateRecorder), the order-perturbed runs `variants` (order_variants), the
    oracle problem P and its unwrapped inner step (classify_flip's probe).  resume (with opt, the
    oracle's options): the GPU state at an outer-iteration head, for forced_outer_flip."""
    exc = []
    env = None

    def reachable(i, j):   # inner step i + 1 wrote log row i + 1
        if i >= len(states):
            return None
        return tcg_exit_reachable(P, states[i], j, max(prefix_deviation(gl, ra.log, i + 2), 1e-14))

    unstable = None
    try:
        if first_branch_flip(gl, ra.log) is not None:
            raise BranchFlip("branches differ")
        env = envelope(ra, variants)
        try:
            compare_logs(gl, ra.log, envelope=env, excursions=exc)
            if gpu_tcg is not None:
                compare_tcg_iters(gpu_tcg, ra, env, reachable=reachable)
        except BranchFlip:
            raise
        except AssertionError:
            # the oracle's own order variants leave the reference's branches at row fv: past it the
            # reference trajectory is not reproducible under summation order (no row-level target),
            # so the rows before fv meet the envelope bar and the outer iterates the inner
            # tolerance (compare_outer), as for a classified flip
            fv = min([f[0] for f in env["_flips"] if f is not None], default=None)
            if fv is None:
                raise
            exc = []
            compare_logs(_prefix(gl, fv), _prefix(ra.log, fv), envelope=env, excursions=exc)
            if gpu_tcg is not None and fv > 1:
                pre = type("Pre", (), {"trace": ra.trace[:fv - 1]})()
                compare_tcg_iters(list(gpu_tcg)[:fv - 1], pre, {"_tcg": env["_tcg"][:fv - 1]}, reachable=reachable)
            compare_outer(gl, ra.log)
            unstable = fv
    except BranchFlip:
        flip = first_branch_flip(gl, ra.log)
        eps = classify_flip(step, P, states, gl, ra.log, flip)
        if eps is None and variant_supports_flip(variants, gl, ra.log, flip):
            eps = 0.0   # the oracle's own summation-order variants leave its branches there (no perturbation)
        if eps is None and decision_tie(step, P, states, gl, ra.log, flip) is not None:
            eps = 0.0   # the decision's margin is inside the evaluation error of ared / pred
        forced = None
        decor = False
        if eps is None and variant_decorrelated(ra, variants, flip):
            eps, decor = 0.0, True
        if eps is None and resume is not None:
            forced = forced_outer_flip(gl, flip, P, opt, resume)
            if forced is not None:
                eps = forced[2]
        if eps is None:
            row = flip[0]
            m = decision_margins(step, P, states[row - 1]) if 1 <= row <= len(states) else None
            raise AssertionError(("branch flip neither reachable within the accumulated drift nor left by the "
                                  "oracle's order variants", flip, gl[flip[1]][row], ra.log[flip[1]][row],
                                  "drift", prefix_deviation(gl, ra.log, row), "margins", m,
                                  "gpu rows", {k: gl[k][max(0, row - 2):row + 2] for k in
                                               ("iteration", "inner_status", "radius_update", "cost", "residual")},
                                  "ref rows", {k: ra.log[k][max(0, row - 2):row + 2] for k in
                                               ("iteration", "inner_status", "radius_update", "cost", "residual")}))
        row = flip[0]
        if forced is None:
            compare_outer(gl, ra.log)
        else:
            # outer-level agreement up to the head of the forced iteration (past it the GPU's rows
            # were checked against the oracle from the GPU's own state)
            head = next(i for i in range(1, len(gl["iteration"])) if gl["iteration"][i] == forced[0]) - 1
            compare_outer(_prefix(gl, head + 1), _prefix(ra.log, head + 1))
            flip = flip + ("forced at outer %d" % forced[0],)
        if decor:
            flip = flip + ("order variants decorrelated before it",)
        # the rows before the flip still meet the envelope bar (and their tCG exit indices)
        if row > 1:
            env = env if env is not None else envelope(ra, variants)
            compare_logs(_prefix(gl, row), _prefix(ra.log, row), envelope=env, excursions=exc)
            if gpu_tcg is not None:
                pre = type("Pre", (), {"trace": ra.trace[:row - 1]})()
                compare_tcg_iters(list(gpu_tcg)[:row - 1], pre, {"_tcg": env["_tcg"][:row - 1]}, reachable=reachable)
        return ("flip", flip[:2] + (eps, len(gl["iteration"]), exc) + flip[2:])
    if unstable is not None:
        return ("unstable", (unstable, exc))
    if gpu_x is not None:
        np.testing.assert_allclose(gpu_x, ra.x, atol=1e-6)
    return ("excursion", exc) if exc else None


def check_instance(gl, Z, x0, y0, opt, gpu_x=None, S=None, gpu_tcg=None):
    """One instance's GPU trajectory against the oracle (dsymv) with tests/parity.py's bar:
    identical branches, outer-iterate values within 1e-4, trial values within 10x the envelope of
    five order-perturbed oracle runs (parity.order_variants / envelope), and the tCG exit index
    of every inner step within the variants' spread (parity.compare_tcg_iters; gpu_tcg = the
    GPU's per-row tCG iterations).  A branch flip must be a classified rounding tie
    (parity.classify_flip: the GPU's decision is reachable from the oracle's own state at that
    step perturbed by at most the outer-iterate drift accumulated before it, capped at 1e-8); the
    trajectories must then still agree at the outer level (parity.compare_outer).
    Returns ("flip", (row, key, eps, rows, excursions)), ("excursion", [(key, rows)]) or None."""
    from oracle import riptrm_oracle as O
    Pa = O.NonnegPCAVectorized(Z, S=S)
    oa = O.RIPTRMOracle(opt)
    rec = StateRecorder(oa)
    ra = oa.run(Pa, x0, y0)
    return check_against(gl, ra, rec.states, order_variants(Z, x0, y0, opt, S=S), Pa, rec.step,
                         gpu_x=gpu_x, gpu_tcg=gpu_tcg)


VARIANT_SEEDS = (1, 2, 6, 7)


def _oracle_job(job):
    """One oracle run in a pool worker (single-threaded BLAS): the reference run with its inner
    steps' starting states recorded, the dgemv variant, or dsymv on a symmetric permutation (the
    runs of check_instance / order_variants)."""
    kind, s_path, x0, y0, opt, seed = job
    from oracle import riptrm_oracle as O
    S = np.load(s_path)
    if kind == "ref":
        oa = O.RIPTRMOracle(opt)
        rec = StateRecorder(oa)
        return oa.run(O.NonnegPCAVectorized(S, S=S), x0, y0), rec.states
    if kind == "gemv":
        return O.RIPTRMOracle(opt).run(O.NonnegPCAVectorized(S, S=S, symv=False), x0, y0), None
    p = np.random.RandomState(seed).permutation(S.shape[0])
    Sp = np.ascontiguousarray(S[p][:, p])
    r = O.RIPTRMOracle(opt).run(O.NonnegPCAVectorized(Sp, S=Sp), x0[p], y0[p])
    inv = np.argsort(p)
    r.x, r.y = np.asarray(r.x)[inv], np.asarray(r.y)[inv]   # back to the instance's own order
    return r, None


def check_instances_parallel(items, opt, workers=16, progress=print, every_s=20.0, null=False):
    """check_instance for many instances with the 6 oracle runs of each (reference + the 5
    order variants) spread over a pool of `workers` single-threaded processes.  items: dicts with
    gl (the GPU log), S (n x n, the device's own S), x0, y0 and optionally gpu_x, gpu_tcg, name.
    Checks run in the parent as each instance's runs complete; `progress(msg)` is called at least
    every `every_s` seconds (long GPU-box tests must show output).  Returns {name: result}."""
    import concurrent.futures as cf
    import multiprocessing as mp
    import os
    import tempfile
    import time
    from oracle import riptrm_oracle as O
    results = {}
    keep = {k: os.environ.get(k) for k in ("OMP_NUM_THREADS", "OPENBLAS_NUM_THREADS", "MKL_NUM_THREADS")}
    with tempfile.TemporaryDirectory() as td:
        paths = []
        for k, it in enumerate(items):
            paths.append(os.path.join(td, f"S{k}.npy"))
            np.save(paths[-1], np.ascontiguousarray(it["S"], dtype=np.float64))
        jobs = {}
        for k, it in enumerate(items):
            args = (paths[k], np.asarray(it["x0"], np.float64), np.asarray(it["y0"], np.float64), opt)
            jobs[(k, "ref")] = ("ref",) + args + (None,)
            jobs[(k, "gemv")] = ("gemv",) + args + (None,)
            for sd in VARIANT_SEEDS:
                jobs[(k, sd)] = ("perm",) + args + (sd,)
        for v in keep:
            os.environ[v] = "1"
        try:
            with cf.ProcessPoolExecutor(max_workers=workers, mp_context=mp.get_context("spawn")) as ex:
                futs = {ex.submit(_oracle_job, j): key for key, j in jobs.items()}
                out, pending, t0, last = {}, set(futs), time.time(), time.time()
                done_items = set()
                while pending:
                    fin, pending = cf.wait(pending, timeout=every_s, return_when=cf.FIRST_COMPLETED)
                    for f in fin:
                        out[futs[f]] = f.result()
                    for k, it in enumerate(items):
                        need = [(k, "ref"), (k, "gemv")] + [(k, sd) for sd in VARIANT_SEEDS]
                        if k in done_items or any(q not in out for q in need):
                            continue
                        done_items.add(k)
                        ra, states = out[(k, "ref")]
                        variants = [out[q][0] for q in need[1:]]
                        S = np.load(paths[k])
                        P = O.NonnegPCAVectorized(S, S=S)
                        name = it.get("name", k)
                        try:
                            if null:
                                r = check_null(it["gl"], ra, variants, it["gpu_x"], it["gpu_y"], it.get("gpu_tcg"))
                            else:
                                r = check_against(it["gl"], ra, states, variants, P, O.RIPTRMOracle(opt).inner_step,
                                                  gpu_x=it.get("gpu_x"), gpu_tcg=it.get("gpu_tcg"),
                                                  resume=it.get("resume"), opt=opt)
                        except AssertionError as e:
                            raise AssertionError((f"instance {name}",) + tuple(e.args)) from e
                        results[name] = r
                        progress(f"[parity] instance {name}: "
                                 + (f"GPU div row {r['gpu']['div_row']} of {r['gpu']['rows']}, variants "
                                    f"{[v['div_row'] for v in r['variants']]}" if null else f"{r}")
                                 + f" ({time.time() - t0:.0f} s)")
                        for q in need:
                            out.pop(q)
                        last = time.time()
                    if time.time() - last >= every_s:
                        progress(f"[parity] {len(done_items)}/{len(items)} instances checked, {len(pending)} oracle runs "
                                 f"pending ({time.time() - t0:.0f} s)")
                        last = time.time()
        finally:
            for v, val in keep.items():
                if val is None:
                    os.environ.pop(v, None)
                else:
                    os.environ[v] = val
    return results


def check_budget(results, B, late_ties_free=False):
    """At most B/2 instances of a test may flip (each a classified rounding tie) and at most
    excursion_budget(B) may show an envelope excursion (before a flip, for flipped ones).
    late_ties_free: flips in the last quarter of an instance's rows reproduced by a perturbation
    <= 1e-12 (the tie regime of small-mu iterations: |normdx - Delta| <= 1e-15 with a tiny Delta,
    RIPTRM.py:672) do not count against the B/2; flips classified by forced_outer_flip (drift-driven:
    the GPU's decision is the oracle's at the GPU's own state) or variant_decorrelated always count."""
    flips = {b: r[1] for b, r in results.items() if r and r[0] == "flip"}
    exc = {b: r[1] for b, r in results.items() if r and r[0] == "excursion"}
    exc.update({b: r[1][1] for b, r in results.items() if r and r[0] == "unstable" and r[1][1]})
    exc.update({b: f[4] for b, f in flips.items() if f[4]})   # flip = (row, key, eps, rows, excursions)
    print("classified flips:", flips, "envelope excursions:", exc)
    counted = {b: f for b, f in flips.items()
               if not (late_ties_free and f[0] >= 0.75 * f[3] and f[2] <= 1e-12 and len(f) < 6)}
    assert len(counted) <= B // 2, flips
    assert len(exc) <= excursion_budget(B), exc


# ---- null calibration: the GPU as one more summation-order variant (round 5) ------------------
#
# The bar above judges the GPU's trajectory against the reference run with classifiers for the
# rows where the two leave each other.  The null test below asks the question those classifiers
# answer indirectly: does the GPU leave the reference run the way a further CPU order variant of
# the same arithmetic does (order_variants: dgemv, dsymv on symmetric permutations), or worse?
# Each run m (the GPU, and every variant) is measured against the reference run R by
#   div_row   the first row whose branch decisions differ (the log length if none);
#   dx, dy    ||x_m - x_R|| and ||y_m - y_R|| / ||y_R|| at the end of the window;
#   outer_dev the largest relative deviation of the KKT residual at the end of each outer iteration.
# Per instance the GPU's dx, dy and outer_dev must be within MULT x the largest variant's (plus a
# rounding floor).  Over the instances of a test, the GPU's divergence row must rank among the
# variants' like one more exchangeable variant: under that null its mid-rank percentile u (0 = it
# diverges before every variant, 1 = after every one) has mean 1/2, and P(u = 0 strictly) <=
# 1/(K+1) per instance; the test fails at level NULL_ALPHA if the mean is too low or there are too
# many strictly-earliest instances.  tests/test_oracle.py calibrates this on the CPU (a variant in
# the GPU's place passes; a run with a 1e-9 relative Hessian error, a real defect far below what a
# trajectory comparison sees by eye, fails).

NULL_MULT = 10.0
NULL_ALPHA = 0.01
NULL_FLOOR_X = 1e-10      # ||x|| = 1: rounding of a K = 20 window is ~1e-13
NULL_FLOOR_Y = 1e-10      # relative
NULL_FLOOR_OUTER = 1e-9   # relative


def outer_residuals(log):
    """{outer iteration k: KKT residual of its last row} (row 0 for k = 0)."""
    it = log["iteration"]
    return {int(it[r]): float(log["residual"][r]) for r in outer_rows(log)}


def run_divergence(log, x, y, ref_log, ref_x, ref_y):
    """One run's distance from the reference run (see above)."""
    f = first_branch_flip(log, ref_log)
    nrows = len(ref_log["iteration"])
    ro, mo = outer_residuals(ref_log), outer_residuals(log)
    ks = sorted(set(ro) & set(mo))
    od = max([abs(mo[k] - ro[k]) / max(abs(ro[k]), 1e-300) for k in ks] + [0.0])
    x, y, rx, ry = (np.asarray(v, float).ravel() for v in (x, y, ref_x, ref_y))
    return {"div_row": nrows if f is None else int(f[0]), "flip": None if f is None else [int(f[0]), f[1]],
            "rows": nrows, "dx": float(np.linalg.norm(x - rx)),
            "dy": float(np.linalg.norm(y - ry) / max(np.linalg.norm(ry), 1e-300)), "outer_dev": float(od)}


def null_row(gpu, variants, mult=NULL_MULT):
    """The GPU's run_divergence against its variants' (a list): mid-rank percentile u of the
    divergence row, whether it is strictly the earliest, and the per-instance bars' ratios."""
    K = len(variants)
    dg = gpu["div_row"]
    below = sum(1 for v in variants if v["div_row"] < dg)
    ties = sum(1 for v in variants if v["div_row"] == dg)
    row = {"gpu": gpu, "variants": variants, "u": (below + 0.5 * ties) / K if K else 0.5,
           "earliest": below == 0 and ties == 0}
    for key, floor in (("dx", NULL_FLOOR_X), ("dy", NULL_FLOOR_Y), ("outer_dev", NULL_FLOOR_OUTER)):
        vmax = max([v[key] for v in variants] + [0.0])
        row[key + "_limit"] = mult * vmax + floor
        row[key + "_ok"] = bool(gpu[key] <= row[key + "_limit"])
    return row


def binom_upper(n, p, alpha):
    """Smallest q with P(Binomial(n, p) > q) <= alpha."""
    from math import comb
    tail = 1.0
    for q in range(n + 1):
        tail -= comb(n, q) * p ** q * (1 - p) ** (n - q)
        if tail <= alpha:
            return q
    return n


def null_summary(rows, alpha=NULL_ALPHA):
    """Aggregate of null_row over a test's instances (see above); ok = every bar holds."""
    from statistics import NormalDist
    n = len(rows)
    K = min(len(r["variants"]) for r in rows)
    mean_u = sum(r["u"] for r in rows) / n
    # the mid-rank of one exchangeable run among K + 1 has variance <= (K + 2) / (12 K) (ties only shrink it)
    sd = ((K + 2) / (12.0 * K * n)) ** 0.5
    u_min = 0.5 - NormalDist().inv_cdf(1 - alpha) * sd
    earliest = sum(1 for r in rows if r["earliest"])
    q = binom_upper(n, 1.0 / (K + 1), alpha)
    per = {k: [i for i, r in enumerate(rows) if not r[k + "_ok"]] for k in ("dx", "dy", "outer_dev")}
    ok = mean_u >= u_min and earliest <= q and not any(per.values())
    return {"instances": n, "variants": K, "mean_u": mean_u, "mean_u_min": u_min, "earliest": earliest,
            "earliest_max": q, "failed_bars": per, "ok": bool(ok)}


def leave_one_out(variant_runs, mult=NULL_MULT):
    """The null's own behaviour: each CPU variant in the GPU's place against the others (K - 1).
    variant_runs: per instance, the list of run_divergence dicts of its K variants.  Returns the
    null_summary of all (instance, variant) rows plus the per-row list."""
    rows = []
    for runs in variant_runs:
        for j in range(len(runs)):
            rows.append(null_row(runs[j], runs[:j] + runs[j + 1:], mult))
    return rows


def check_null(gl, ra, variants, gpu_x, gpu_y, gpu_tcg=None):
    """One instance's GPU trajectory under the round-5 bar: the rows on which the reference run is
    reproducible under summation order (before every variant's first branch flip) and before the
    GPU's own first flip meet the envelope bar (compare_logs(envelope=...), compare_tcg_iters);
    past them the trajectory is summarised by run_divergence, against the variants', in null_row
    (the per-instance MULT bars here, the rank test over the instances in null_summary).  Returns
    the null_row dict (+ the envelope excursions and the number of rows compared row by row)."""
    env = envelope(ra, variants)
    nrows = len(ra.log["iteration"])
    fv = min([f[0] for f in env["_flips"] if f is not None], default=nrows)
    fg = first_branch_flip(gl, ra.log)
    upto = min(fv, nrows if fg is None else fg[0])
    exc = []
    if upto > 0:
        compare_logs(_prefix(gl, upto), _prefix(ra.log, upto), envelope=env, excursions=exc)
    if gpu_tcg is not None and upto > 1:
        pre = type("Pre", (), {"trace": ra.trace[:upto - 1]})()
        compare_tcg_iters(list(gpu_tcg)[:upto - 1], pre, {"_tcg": env["_tcg"][:upto - 1]})
    vr = [run_divergence(v.log, v.x, v.y, ra.log, ra.x, ra.y) for v in variants]
    row = null_row(run_divergence(gl, gpu_x, gpu_y, ra.log, ra.x, ra.y), vr)
    row.update(excursions=exc, rows_compared=int(upto))
    return row


def null_table(rows, names, summary, path=None):
    """The per-instance table of a null test (GPU vs variants: divergence rows, final distances,
    outer deviation) as JSON-able dict; written to `path` when given."""
    import json
    out = {"summary": summary, "instances": []}
    for name, r in zip(names, rows):
        g = r["gpu"]
        out["instances"].append({
            "name": name, "rows": g["rows"], "gpu_first_flip": g["flip"], "gpu_div_row": g["div_row"],
            "variant_div_rows": [v["div_row"] for v in r["variants"]], "u": r["u"], "earliest": r["earliest"],
            "gpu_dx": g["dx"], "variant_dx_max": max(v["dx"] for v in r["variants"]),
            "gpu_dy": g["dy"], "variant_dy_max": max(v["dy"] for v in r["variants"]),
            "gpu_outer_dev": g["outer_dev"], "variant_outer_dev_max": max(v["outer_dev"] for v in r["variants"]),
            "rows_compared_row_by_row": r.get("rows_compared"), "excursions": r.get("excursions")})
    if path:
        import os
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        json.dump(out, open(path, "w"), indent=1, default=str)
    return out


def assert_null(rows, names, path=None, budget=None):
    """null_summary over a test's rows; the table goes to `path`; fails on any bar (and on more
    envelope excursions than excursion_budget)."""
    summary = null_summary(rows)
    tab = null_table(rows, names, summary, path)
    for it in tab["instances"]:
        print("[null]", it["name"], "gpu div row", it["gpu_div_row"], "of", it["rows"], "variants", it["variant_div_rows"],
              "u %.2f" % it["u"], "dx %.1e (variants %.1e)" % (it["gpu_dx"], it["variant_dx_max"]),
              "outer %.1e (%.1e)" % (it["gpu_outer_dev"], it["variant_outer_dev_max"]), flush=True)
    print("[null] summary", summary, flush=True)
    exc = [n for n, r in zip(names, rows) if r.get("excursions")]
    assert len(exc) <= (excursion_budget(len(rows)) if budget is None else budget), exc
    assert summary["ok"], summary
    return summary


def si_order_variants(data, x0, y0, opt, seeds=(1, 2, 3), structured=True):
    """StableIdentification runs that are the same arithmetic in another summation order: the
    reference-structured wiring (SIStructured: per-constraint loops, RIPTRM.py:475-571), and the
    vectorised oracle on a coordinate permutation Pi (X, XP -> Pi X, Pi XP; J, R, Q -> Pi J Pi^T ...;
    the constraints on A_rc -> A'_{pi(r) pi(c)}, their order shuffled too), which leaves the cost,
    the constraints, the SPD metric and every logged quantity invariant (A' = Pi A Pi^T, E' = Pi E).
    x and y of the permuted runs are mapped back.  The SI analogue of order_variants."""
    import copy
    from oracle import si_oracle as SI
    out = []
    if structured:
        out.append(SI.solve(data, x0, y0, opt, structured=True))
    d, m = data.d, data.m
    for sd in seeds:
        rs = np.random.RandomState(sd)
        p = rs.permutation(d)
        inv = np.argsort(p)
        sig = rs.permutation(m)
        dp = copy.copy(data)
        dp.X, dp.XP = np.ascontiguousarray(data.X[p]), np.ascontiguousarray(data.XP[p])
        dp.cons = [(k, int(inv[r]), int(inv[c]), p0, p1) for (k, r, c, p0, p1) in (data.cons[i] for i in sig)]
        xp = np.stack([np.asarray(x0)[k][p][:, p] for k in range(3)])
        r = SI.solve(dp, xp, np.asarray(y0)[sig], opt)
        r.x = np.stack([np.asarray(r.x)[k][inv][:, inv] for k in range(3)])
        yy = np.empty(m)
        yy[sig] = np.asarray(r.y)
        r.y = yy
        out.append(r)
    return out
