"""Generates tests/golden/si_1_pins/oracle_minres.json: the CPU oracle's (oracle/si_oracle.py,
SIVectorized) per-start minimum log10 KKT residual on the reference fixture
dataset/StableIdentification/1 under the protocol the pin tests use, next to the values the
reference itself published (src/StableIdentification/analyzer.ipynb, box-plot cell: per-start
min over the log of the 240 s run, log10; printed rows and quartiles).

  RIPTRM (tCG):   maxiter 35, inner_maxiter 300 (the outer loop stalls at mu ~ 3e-14 once the
                  inner tolerance max(mu, 1e-14) is out of reach; the reference ran into its
                  240 s limit there instead)
  RIPTRM (exact): Exact_RepMat + second-order test, maxiter 25, inner_maxiter 300 (the reference's
                  exact runs stall inside outer iteration 25, mu_25 = 4.08e-10, at residual
                  4 mu_25 for every start)

Run: python tests/golden/make_si_pins.py  (about 10 minutes on one core)."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import si_oracle as SI  # noqa: E402

DS = os.path.join(ROOT, "tests", "golden", "si_1")
PTS = "abcdefghijklmnopqrst"
PUBLISHED = {
    "source": "src/StableIdentification/analyzer.ipynb, box-plot cell output",
    "tcg_start_t": -12.475348,
    "tcg_quartiles": [-12.444660, -12.368153, -12.225336],
    "exact_every_start": -8.787497,
}
TCG = dict(tolresid=0.0, maxtime=1e9, maxiter=35, inner_maxiter=300)
EXACT = dict(tolresid=0.0, maxtime=1e9, maxiter=25, inner_maxiter=300, TRS_solver="Exact_RepMat",
             second_order_stationarity=True)


def min_log_res(pt, opt):
    data = SI.SIData.load(DS)
    x0, y0 = SI.load_start(DS, pt)
    ref = SI.solve(data, x0, y0, dict(opt, manviofun=SI.si_manvio))
    r = np.array(ref.log["residual"], float)
    it = np.array(ref.log["iteration"])
    return float(np.log10(r.min())), int(it[r.argmin()])


def main():
    out = {"published": PUBLISHED, "protocol": {"tcg": TCG, "exact": EXACT},
           "tcg": {p: min_log_res(p, TCG) for p in PTS},
           "exact": {p: min_log_res(p, EXACT) for p in "at"}}
    v = np.array([out["tcg"][p][0] for p in PTS])
    out["tcg_quartiles"] = [float(np.quantile(v, 0.25)), float(np.median(v)), float(np.quantile(v, 0.75))]
    path = os.path.join(ROOT, "tests", "golden", "si_1_pins", "oracle_minres.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out["tcg_quartiles"]), out["exact"])


if __name__ == "__main__":
    main()
