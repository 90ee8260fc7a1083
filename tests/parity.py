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
"""
import numpy as np

BRANCH_KEYS = ("iteration", "num_inner", "inner_status", "dxtype", "radius_update", "dual_clipping")
VALUE_KEYS = ("residual", "cost", "gradnorm", "complviolation", "dualviolation", "manviolation",
              "maxviolation", "meanviolation", "mu", "normdx", "TR_radius", "minxfeasi", "minyfeasi",
              "compl", "ared/pred", "maxabsLagmult")
# properties of the tCG step / trial point rather than of the iterate: trial bounds on every row
STEP_KEYS = ("normdx", "minxfeasi", "minyfeasi", "compl", "ared/pred")


def _col(log, k):
    return np.array([np.nan if v is None else float(v) for v in log[k]], dtype=float)


def compare_logs(gl, rl, rtol=1e-4, ascale=1e-5, trial_rtol=1.0, trial_ascale=1e-2, atol=1e-14):
    assert list(gl.keys()) == list(rl.keys()), (list(gl.keys()), list(rl.keys()))
    assert len(gl["iteration"]) == len(rl["iteration"]), (len(gl["iteration"]), len(rl["iteration"]))
    for k in BRANCH_KEYS:
        if k in gl:
            assert gl[k] == rl[k], k
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
        rows_outer = outer if k not in STEP_KEYS else np.zeros_like(outer)
        bad = m & np.where(rows_outer, ~ok_outer, ~ok_trial)
        assert not bad.any(), (k, np.nonzero(bad)[0][:5], g[bad][:5], r[bad][:5])
