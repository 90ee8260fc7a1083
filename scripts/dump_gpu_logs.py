"""GPU trajectories for offline parity analysis (tests/parity.py's null-calibrated bar is developed on
the CPU against these): NonnegPCA instances drawn by the host generator (oracle/nonnegpca_gen.py,
seeds seed0 .. seed0 + B - 1), solved on the device over K outer iterations with the bench window's
options, then per instance the log (the reference's columns), the tCG iterations per row and the
final x, y are written to OUT (JSON + .npz).

    python scripts/dump_gpu_logs.py OUT N B K SEED0
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "riemannian-interior-point-trust-region-method_amd")]


def _plain(v):
    if v is None or isinstance(v, (str, bool, int)):
        return v
    if isinstance(v, np.bool_):
        return bool(v)
    if isinstance(v, np.integer):
        return int(v)
    return float(v)


def main():
    out, n, B, K, seed0 = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])
    import engine
    from oracle import nonnegpca_gen as G
    from problems import manviofun
    os.makedirs(out, exist_ok=True)
    eng = engine.NonnegPCABatch(n, B)
    Zs, xs, ys = [], [], []
    for b in range(B):
        Z, x0, y0 = G.generate_instance(n, seed0 + b)
        Zs.append(Z)
        xs.append(x0)
        ys.append(y0)
    eng.load_Z(np.stack(Zs))
    del Zs
    opt = {"TRS_solver": "tCG", "second_order_stationarity": False, "manviofun": manviofun,
           "tolresid": 0.0, "maxtime": 1e9, "maxiter": K}
    res = eng.solve(np.stack(xs), np.stack(ys), opt)
    print(f"solved {B} instances n={n} K={K}", flush=True)
    logs = []
    for b in range(B):
        gl = res.log(b)
        logs.append({"seed": seed0 + b, "log": {k: [_plain(v) for v in col] for k, col in gl.items()},
                     "tcg": res.tcg_iters_per_row(b)[1:], "outer": int(res.stat(b, "OUTER_ITERS"))})
    json.dump({"n": n, "K": K, "seed0": seed0, "instances": logs}, open(os.path.join(out, "logs.json"), "w"))
    np.savez(os.path.join(out, "xy.npz"), x=res.x.cpu().numpy()[:, :n], y=res.y.cpu().numpy()[:, :n])
    print("wrote", out, flush=True)


if __name__ == "__main__":
    main()
