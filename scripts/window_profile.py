"""Per-outer-iteration cost of the batched GPU solve (S-passes, tCG iterations, seconds)."""
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "riemannian-interior-point-trust-region-method_amd")]

import torch  # noqa: E402

import engine  # noqa: E402
from problems import manviofun  # noqa: E402


def main():
    n, B, K = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
    torch.cuda.set_device(0)
    eng = engine.NonnegPCABatch(n, B, log_capacity=8192)
    x0, y0 = eng.generate_synthetic()
    opt = {"TRS_solver": "tCG", "maxiter": K, "tolresid": 0.0, "maxtime": math.inf, "manviofun": manviofun}
    eng.begin(x0, y0, opt)
    C = engine.C
    prev = eng.stats()
    t_all = time.perf_counter()
    for k in range(1, K + 1):
        t0 = time.perf_counter()
        eng.run_until(k)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        st = eng.stats()
        dp = st - prev
        prev = st
        row = {"n": n, "B": B, "outer": k, "sec": dt,
               "passes_sum": float(dp[:, C["RIPTRM_STAT_PASSES"]].sum()),
               "passes_max": float(dp[:, C["RIPTRM_STAT_PASSES"]].max()),
               "tcg_sum": float(dp[:, C["RIPTRM_STAT_TCG_ITERS"]].sum()),
               "inner_sum": float(dp[:, C["RIPTRM_STAT_INNER_ITERS"]].sum())}
        print(json.dumps(row), flush=True)
    print(json.dumps({"n": n, "B": B, "total_sec": time.perf_counter() - t_all}), flush=True)


if __name__ == "__main__":
    main()
