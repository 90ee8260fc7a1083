"""Diagnostic (GPU): the full log of the Exact_RepMat StableIdentification solve of one fixture
start (maxiter / inner_maxiter as the pin protocol), as JSON, for a row-by-row comparison with
the CPU oracle."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "riemannian-interior-point-trust-region-method_amd")]
import si  # noqa: E402
from oracle import si_oracle as SI  # noqa: E402

DS = os.path.join(ROOT, "tests", "golden", "si_1")
data = SI.SIData.load(DS)
pt = sys.argv[1] if len(sys.argv) > 1 else "a"
maxiter = int(sys.argv[2]) if len(sys.argv) > 2 else 25
x0, y0 = SI.load_start(DS, pt)
eng = si.SIBatch(data.d, data.N, data.m, 1, log_capacity=8192)
eng.load(data.X, data.XP, data.h, si.expand_constset(np.loadtxt(os.path.join(DS, "constset.csv"))))
res = eng.solve(x0[None], y0[None], {"TRS_solver": "Exact_RepMat", "second_order_stationarity": True,
                                     "manviofun": si.si_manviofun, "tolresid": 0.0, "maxtime": 1e9,
                                     "maxiter": maxiter, "inner_maxiter": 300})
lg = res.log(0)
print(json.dumps({k: [None if v is None else (v if isinstance(v, str) else float(v)) for v in lg[k]] for k in lg}))
