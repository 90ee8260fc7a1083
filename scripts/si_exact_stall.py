"""Diagnostic (GPU): the Exact_RepMat StableIdentification run on fixture start a, outer iteration
25 (where the reference's exact runs stall at residual 4 mu_25): the residual / inner status /
radius / step norm of every row there, next to the CPU oracle's (tests/golden/si_1_pins protocol)."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "riemannian-interior-point-trust-region-method_amd"), os.path.join(ROOT, "tests")]
import si  # noqa: E402
from oracle import si_oracle as SI  # noqa: E402

DS = os.path.join(ROOT, "tests", "golden", "si_1")
data = SI.SIData.load(DS)
pt = sys.argv[1] if len(sys.argv) > 1 else "a"
x0, y0 = SI.load_start(DS, pt)
eng = si.SIBatch(data.d, data.N, data.m, 1, log_capacity=8192)
eng.load(data.X, data.XP, data.h, si.expand_constset(np.loadtxt(os.path.join(DS, "constset.csv"))))
res = eng.solve(x0[None], y0[None], {"TRS_solver": "Exact_RepMat", "second_order_stationarity": True,
                                     "manviofun": si.si_manviofun, "tolresid": 0.0, "maxtime": 1e9,
                                     "maxiter": 25, "inner_maxiter": 300})
lg = res.log(0)
it = np.array(lg["iteration"])
r = np.array(lg["residual"], float)
rows = np.nonzero(it >= 24)[0]
out = {"rows": int(len(r)), "min_log10": float(np.log10(r.min())), "argmin_row": int(r.argmin()),
       "iter25": [[int(i), lg["inner_status"][i], float(r[i]), lg["radius_update"][i], lg["dxtype"][i],
                   None if lg["normdx"][i] is None else float(lg["normdx"][i]),
                   None if lg["TR_radius"][i] is None else float(lg["TR_radius"][i]),
                   None if lg["mineigvalHw"][i] is None else float(lg["mineigvalHw"][i])] for i in rows[:80]]}
print(json.dumps(out))
