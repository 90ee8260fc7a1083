"""Diagnostic (GPU): per-instance trajectory deviations of the HIP path from the vectorised oracle,
next to the deviations between two CPU oracles that differ only in the S.v summation order
(dsymv vs dgemv): first branch flip, and per quantity the max relative deviation on outer rows and
on trial rows.  Used to calibrate tests/parity.py."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "riemannian-interior-point-trust-region-method_amd"), os.path.join(ROOT, "tests")]
import engine  # noqa: E402
from oracle import nonnegpca_gen as G  # noqa: E402
from oracle import riptrm_oracle as O  # noqa: E402
from parity import VALUE_KEYS, _col, first_branch_flip  # noqa: E402
from problems import manviofun  # noqa: E402

OPT = dict(tolresid=0.0, maxtime=1e9)


def dev(a, b):
    out = {}
    outer = np.array([s in (None, "converged") for s in b["inner_status"]])
    for k in VALUE_KEYS:
        if k not in a or k not in b:
            continue
        m = min(len(a[k]), len(b[k]))
        g, r = _col(a, k)[:m], _col(b, k)[:m]
        ok = ~np.isnan(r) & ~np.isnan(g)
        if not ok.any():
            continue
        scale = np.max(np.abs(r[ok])) or 1.0
        rel = np.abs(g - r) / np.maximum(np.abs(r), 1e-12 * scale)
        o = rel[ok & outer[:m]]
        t = rel[ok & ~outer[:m]]
        out[k] = [float(o.max()) if o.size else 0.0, float(t.max()) if t.size else 0.0]
    return out


def main():
    cases = [(37, 5, 10, 100), (200, 4, 12, 100), (1000, 2, 10, 100), (300, 3, 10, 100), (4000, 2, 12, 4000)]
    for n, B, K, s0 in cases:
        insts = [G.generate_instance(n, s0 + b) for b in range(B)]
        eng = engine.NonnegPCABatch(n, B, log_capacity=4096)
        eng.load_Z(np.stack([z for z, _, _ in insts]))
        res = eng.solve(np.stack([x for _, x, _ in insts]), np.stack([y for _, _, y in insts]),
                        {"TRS_solver": "tCG", "second_order_stationarity": False, "manviofun": manviofun,
                         "maxiter": K, **OPT})
        for b, (Z, x0, y0) in enumerate(insts):
            o = dict(OPT, maxiter=K, manviofun=O.sphere_manvio)
            a = O.RIPTRMOracle(o).run(O.NonnegPCAVectorized(Z, symv=True), x0, y0)
            c = O.RIPTRMOracle(o).run(O.NonnegPCAVectorized(Z, symv=False), x0, y0)
            gl = res.log(b)
            print(json.dumps({"n": n, "b": b, "seed": s0 + b, "rows": [len(gl["iteration"]), len(a.log["iteration"])],
                              "flip_gpu": first_branch_flip(gl, a.log), "flip_cpu_pair": first_branch_flip(c.log, a.log),
                              "dev_gpu": dev(gl, a.log), "dev_cpu_pair": dev(c.log, a.log)}), flush=True)


if __name__ == "__main__":
    main()
