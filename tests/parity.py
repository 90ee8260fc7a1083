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

Round 5: that row-by-row bar applies only where it is meaningful -- on the rows before the
reference run's first order-sensitive row (any order variant's first branch flip) and before the
GPU's own first flip.  Over the whole window the GPU must leave the reference run like one more
order variant (check_null / null_summary below, calibrated on the CPU by
tests/test_oracle.py::test_null_calibration_accepts_variants_and_rejects_hessian_error).  This
replaces round 4's post-hoc flip classifiers (perturbation reachability, decision ties, variant
support, decorrelation, forced outer restarts), which decided case by case whether a flip was
"rounding-driven".
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
        r = O.RIPTRMOracle(option).run(O.NonnegPCAVectorized(Sp, S=Sp), x0[p], y0[p])
        inv = np.argsort(p)
        r.x, r.y = np.asarray(r.x)[inv], np.asarray(r.y)[inv]   # back to the instance's own order
        out.append(r)
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


def compare_tcg_iters(g_iters, ref, env, mult=3.0, rel=0.005, slack=2):
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
    assert not bad.any(), (np.nonzero(bad)[0][:5], g[bad][:5], r[bad][:5], djmax)
    moved = int(np.sum(g != r))
    assert abs(g.sum() - r.sum()) <= max(slack * moved, mult * djmax * moved, rel * r.sum()), (g.sum(), r.sum())


def column_deviation(a, r, k):
    """max over rows of |a - r| / max(|r|, 1e-12 max|r|) for column k (rows both logs have)."""
    m = min(len(a[k]), len(r[k]))
    g, v = _col(a, k)[:m], _col(r, k)[:m]
    ok = ~np.isnan(g) & ~np.isnan(v)
    if not ok.any():
        return 0.0
    scale = np.max(np.abs(v[ok])) or 1.0
    return float(np.max(np.abs(g[ok] - v[ok]) / np.maximum(np.abs(v[ok]), 1e-12 * scale)))


def check_instance(gl, Z, x0, y0, opt, gpu_x, gpu_y, S=None, gpu_tcg=None):
    """One instance's GPU trajectory against the oracle (dsymv) and its five order variants
    (order_variants) under check_null's bar; returns the null_row (the caller pools a test's rows
    in assert_null)."""
    from oracle import riptrm_oracle as O
    ra = O.RIPTRMOracle(opt).run(O.NonnegPCAVectorized(Z, S=S), x0, y0)
    return check_null(gl, ra, order_variants(Z, x0, y0, opt, S=S), gpu_x, gpu_y, gpu_tcg)


VARIANT_SEEDS = (1, 2, 6, 7)


def _oracle_job(job):
    """One oracle run in a pool worker (single-threaded BLAS): the reference run, the dgemv
    variant, or dsymv on a symmetric permutation (the runs of check_instance / order_variants)."""
    kind, s_path, x0, y0, opt, seed = job
    from oracle import riptrm_oracle as O
    S = np.load(s_path)
    if kind == "ref":
        return O.RIPTRMOracle(opt).run(O.NonnegPCAVectorized(S, S=S), x0, y0), None
    if kind == "gemv":
        return O.RIPTRMOracle(opt).run(O.NonnegPCAVectorized(S, S=S, symv=False), x0, y0), None
    p = np.random.RandomState(seed).permutation(S.shape[0])
    Sp = np.ascontiguousarray(S[p][:, p])
    r = O.RIPTRMOracle(opt).run(O.NonnegPCAVectorized(Sp, S=Sp), x0[p], y0[p])
    inv = np.argsort(p)
    r.x, r.y = np.asarray(r.x)[inv], np.asarray(r.y)[inv]   # back to the instance's own order
    return r, None


def check_instances_parallel(items, opt, workers=16, progress=print, every_s=20.0):
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
                        ra = out[(k, "ref")][0]
                        variants = [out[q][0] for q in need[1:]]
                        name = it.get("name", k)
                        try:
                            r = check_null(it["gl"], ra, variants, it["gpu_x"], it["gpu_y"], it.get("gpu_tcg"))
                        except AssertionError as e:
                            raise AssertionError((f"instance {name}",) + tuple(e.args)) from e
                        results[name] = r
                        progress(f"[parity] instance {name}: GPU div row {r['gpu']['div_row']} of {r['gpu']['rows']}, "
                                 f"variants {[v['div_row'] for v in r['variants']]} ({time.time() - t0:.0f} s)")
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

NULL_MULT = 100.0         # per-instance gross bar (the rank tests below carry the calibrated claim)
NULL_ALPHA = 0.01         # family-wise level of the four rank statistics
NULL_FLOOR_X = 1e-8       # ||x|| = 1; a late-window branch flip moves x by ~1e-9 at n = 4000
NULL_FLOOR_Y = 1e-8       # relative
NULL_FLOOR_OUTER = 1e-6   # relative
NULL_KEYS = ("div_row", "dx", "dy", "outer_dev")   # div_row: earlier is worse; the others: larger is worse
NULL_U_MIN_FLOOR = 0.2    # a pooled rank test's mean-u limit must exceed this (assert_null)


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


def _worse(key, v, g):
    return v < g if key == "div_row" else v > g


def null_row(gpu, variants, mult=NULL_MULT):
    """The GPU's run_divergence against its K variants' (a list).  Per statistic of NULL_KEYS: u =
    the fraction of variants that are worse than the GPU (ties count half; 0 = the GPU is the worst
    of the K + 1 runs, 1/2 = the middle, as one more exchangeable variant would be on average) and
    whether the GPU is strictly the worst; per instance the gross bar: each distance within
    `mult` x the farthest variant's plus a rounding floor."""
    K = len(variants)
    row = {"gpu": gpu, "variants": variants}
    for key in NULL_KEYS:
        worse = sum(1 for v in variants if _worse(key, v[key], gpu[key]))
        ties = sum(1 for v in variants if v[key] == gpu[key])
        row["u_" + key] = (worse + 0.5 * ties) / K if K else 0.5
        row["worst_" + key] = worse == 0 and ties == 0
    row["u"], row["earliest"] = row["u_div_row"], row["worst_div_row"]
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
    """Aggregate of null_row over a test's instances; ok = every bar holds.  For each statistic of
    NULL_KEYS, at level alpha / 4 each: the mean of u must not fall below 1/2 by more than the
    normal quantile times its null standard deviation (the mid-rank of one exchangeable run among
    K + 1 has variance <= (K + 2) / (12 K); ties only shrink it), and the number of instances where
    the GPU is strictly the worst must not exceed the Binomial(n, 1 / (K + 1)) upper quantile."""
    from statistics import NormalDist
    n = len(rows)
    K = min(len(r["variants"]) for r in rows)
    a = alpha / len(NULL_KEYS)
    sd = ((K + 2) / (12.0 * K * n)) ** 0.5
    u_min = 0.5 - NormalDist().inv_cdf(1 - a) * sd
    q = binom_upper(n, 1.0 / (K + 1), a)
    stats, ok = {}, True
    for key in NULL_KEYS:
        mean_u = sum(r["u_" + key] for r in rows) / n
        worst = sum(1 for r in rows if r["worst_" + key])
        good = mean_u >= u_min and worst <= q
        stats[key] = {"mean_u": mean_u, "worst": worst, "ok": bool(good)}
        ok = ok and good
    gross = {k: [i for i, r in enumerate(rows) if not r[k + "_ok"]] for k in ("dx", "dy", "outer_dev")}
    ok = ok and not any(gross.values())
    return {"instances": n, "variants": K, "mean_u_min": u_min, "worst_max": q, "stats": stats,
            "mean_u": stats["div_row"]["mean_u"], "earliest": stats["div_row"]["worst"],
            "failed_gross_bars": gross, "ok": bool(ok)}


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
            "variant_div_rows": [v["div_row"] for v in r["variants"]],
            "variant_first_flips": [v["flip"] for v in r["variants"]],
            "u": {k: r["u_" + k] for k in NULL_KEYS}, "gpu_worst": [k for k in NULL_KEYS if r["worst_" + k]],
            "gpu_dx": g["dx"], "variant_dx_max": max(v["dx"] for v in r["variants"]),
            "gpu_dy": g["dy"], "variant_dy_max": max(v["dy"] for v in r["variants"]),
            "gpu_outer_dev": g["outer_dev"], "variant_outer_dev_max": max(v["outer_dev"] for v in r["variants"]),
            "rows_compared_row_by_row": r.get("rows_compared"), "excursions": r.get("excursions")})
    if path:
        import os
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        json.dump(out, open(path, "w"), indent=1, default=str)
    return out


def assert_null(rows, names, path=None, budget=None, variants_move=False):
    """null_summary over a test's rows; the table goes to `path`; fails on any bar (and on more
    envelope excursions than excursion_budget).  A rank test over too few instances cannot fail
    (its mean-u limit sinks towards 0: 0.11 at 6 instances with 5 variants), so a test must pool
    enough instances that the limit exceeds NULL_U_MIN_FLOOR (11 with 4 or 5 variants); the power
    of the bar at those sizes is tests/test_oracle.py::test_null_calibration_accepts_variants_and_rejects_hessian_error.
    variants_move: every instance's variants must end away from the reference run (dx, dy > 0),
    so that the final-point statistics are not vacuous (a window that ends at the start point)."""
    summary = null_summary(rows)
    assert summary["mean_u_min"] > NULL_U_MIN_FLOOR, ("too few instances for the rank test", summary["instances"],
                                                      summary["variants"], summary["mean_u_min"])
    if variants_move:
        still = [n for n, r in zip(names, rows)
                 if max(v["dx"] for v in r["variants"]) <= 0.0 or max(v["dy"] for v in r["variants"]) <= 0.0]
        assert not still, ("variants end at the reference run's final point: vacuous dx / dy", still)
    tab = null_table(rows, names, summary, path)
    for it in tab["instances"]:
        print("[null]", it["name"], "gpu div row", it["gpu_div_row"], "of", it["rows"], "variants", it["variant_div_rows"],
              "u %s" % {k: round(v, 2) for k, v in it["u"].items()}, "dx %.1e (variants %.1e)" % (it["gpu_dx"], it["variant_dx_max"]),
              "outer %.1e (%.1e)" % (it["gpu_outer_dev"], it["variant_outer_dev_max"]), flush=True)
    print("[null] summary", summary, flush=True)
    exc = [n for n, r in zip(names, rows) if r.get("excursions")]
    assert len(exc) <= (excursion_budget(len(rows)) if budget is None else budget), exc
    assert summary["ok"], summary
    return summary


def si_variant(data, x0, y0, opt, which):
    """One StableIdentification run of the oracle: which = "ref" (the vectorised oracle, the
    reference run R), "structured" (the reference-structured wiring, SIStructured: per-constraint
    loops, RIPTRM.py:475-571) or an int seed: the vectorised oracle on a coordinate permutation Pi
    (X, XP -> Pi X, Pi XP; J, R, Q -> Pi J Pi^T ...; the constraints on A_rc -> A'_{pi(r) pi(c)}, their
    order shuffled too), which leaves the cost, the constraints, the SPD metric and every logged
    quantity invariant (A' = Pi A Pi^T, E' = Pi E); x and y of a permuted run are mapped back."""
    import copy
    from oracle import si_oracle as SI
    if which == "ref":
        return SI.solve(data, x0, y0, opt)
    if which == "structured":
        return SI.solve(data, x0, y0, opt, structured=True)
    d, m = data.d, data.m
    rs = np.random.RandomState(int(which))
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
    return r


def si_order_variants(data, x0, y0, opt, seeds=(1, 2, 3), structured=True):
    """StableIdentification runs that are the same arithmetic in another summation order
    (si_variant): the reference-structured wiring and coordinate / constraint-order permutations.
    The SI analogue of order_variants."""
    return [si_variant(data, x0, y0, opt, w) for w in ((["structured"] if structured else []) + list(seeds))]


def _si_job(job):
    data, x0, y0, opt, which = job
    from oracle import si_oracle as SI
    opt = dict(opt, manviofun=SI.si_manvio)
    return si_variant(data, x0, y0, opt, which)


def check_si_parallel(items, workers=16, progress=print, every_s=20.0):
    """check_null for StableIdentification instances with the oracle runs (the reference run and the
    variants `item["variants"]`, a list of si_variant `which` values) spread over a pool of
    single-threaded processes.  items: dicts with data (SIData), x0, y0, opt (without manviofun),
    gl (the GPU log), gpu_x (3 x d x d), gpu_y, variants, name.  Returns {name: null_row}."""
    import concurrent.futures as cf
    import multiprocessing as mp
    import os
    import time
    keep = {k: os.environ.get(k) for k in ("OMP_NUM_THREADS", "OPENBLAS_NUM_THREADS", "MKL_NUM_THREADS")}
    results = {}
    for v in keep:
        os.environ[v] = "1"
    try:
        with cf.ProcessPoolExecutor(max_workers=workers, mp_context=mp.get_context("spawn")) as ex:
            futs = {}
            # the longest runs first (items in the order given; callers list the large d first)
            for k, it in enumerate(items):
                for w in ["ref"] + list(it["variants"]):
                    futs[ex.submit(_si_job, (it["data"], it["x0"], it["y0"], it["opt"], w))] = (k, w)
            out, pending, t0, last = {}, set(futs), time.time(), time.time()
            done = set()
            while pending:
                fin, pending = cf.wait(pending, timeout=every_s, return_when=cf.FIRST_COMPLETED)
                for f in fin:
                    out[futs[f]] = f.result()
                for k, it in enumerate(items):
                    need = [(k, w) for w in ["ref"] + list(it["variants"])]
                    if k in done or any(q not in out for q in need):
                        continue
                    done.add(k)
                    ra, vs = out[need[0]], [out[q] for q in need[1:]]
                    try:
                        r = check_null(it["gl"], ra, vs, it["gpu_x"], it["gpu_y"])
                    except AssertionError as e:
                        raise AssertionError((f"instance {it['name']}",) + tuple(e.args)) from e
                    r["ref_residual0"] = float(ra.log["residual"][0])
                    results[it["name"]] = r
                    progress(f"[si null] {it['name']}: GPU div row {r['gpu']['div_row']} of {r['gpu']['rows']}, "
                             f"variants {[v['div_row'] for v in r['variants']]} ({time.time() - t0:.0f} s)")
                    for q in need:
                        out.pop(q)
                    last = time.time()
                if time.time() - last >= every_s:
                    progress(f"[si null] {len(done)}/{len(items)} instances checked, {len(pending)} oracle runs pending "
                             f"({time.time() - t0:.0f} s)")
                    last = time.time()
    finally:
        for v, val in keep.items():
            if val is None:
                os.environ.pop(v, None)
            else:
                os.environ[v] = val
    return results
