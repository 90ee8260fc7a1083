"""Diagnostic (GPU): step a small persistent solve launch by launch and print each instance's
phase / counters (to localise a non-progressing persistent run)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "riemannian-interior-point-trust-region-method_amd")]
import engine  # noqa: E402
from oracle import nonnegpca_gen as G  # noqa: E402
from problems import manviofun  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 37
B = int(sys.argv[2]) if len(sys.argv) > 2 else 1
mode = int(sys.argv[3]) if len(sys.argv) > 3 else 1
insts = [G.generate_instance(n, 900 + b) for b in range(B)]
eng = engine.NonnegPCABatch(n, B, log_capacity=4096, persistent=mode)
eng.load_Z(np.stack([z for z, _, _ in insts]))
eng.begin(np.stack([x for _, x, _ in insts]), np.stack([y for _, _, y in insts]),
          {"maxiter": int(sys.argv[4]) if len(sys.argv) > 4 else 3, "tolresid": 0.0, "maxtime": 1e9, "manviofun": manviofun, "TRS_solver": "tCG",
           "second_order_stationarity": False})
C = engine.C
act = eng.advance(0)
print("advance(0) ->", act, eng.persistent_state(), flush=True)
for it in range(int(sys.argv[5]) if len(sys.argv) > 5 else 40):
    act = eng.advance(4)
    st = eng.stats()
    print(it, "act", act, "phase", st[:, C["RIPTRM_STAT_PHASE"]].tolist(), "outer", st[:, C["RIPTRM_STAT_OUTER_ITERS"]].tolist(),
          "passes", st[:, C["RIPTRM_STAT_PASSES"]].tolist(), "tcg", st[:, C["RIPTRM_STAT_TCG_ITERS"]].tolist(),
          "err", st[:, C["RIPTRM_STAT_ERROR"]].tolist(), flush=True)
    if act == 0:
        break
