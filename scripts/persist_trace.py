"""Diagnostic (GPU): per-step timing of k_persist (riptrm_persist_trace) at BASELINE configs[1]
(n = 1000, one instance): tile pass, barrier wait, state step, in microseconds of the device clock."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "riemannian-interior-point-trust-region-method_amd")]
import engine  # noqa: E402
from problems import manviofun  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
B = int(sys.argv[2]) if len(sys.argv) > 2 else 1
cap = 256
eng = engine.NonnegPCABatch(n, B, log_capacity=2048, drain_logs=False)
x0, y0 = eng.generate_synthetic()
buf = torch.zeros((2, cap, 24), dtype=torch.int64, device=eng.device)
eng.ctx.check(eng.lib.riptrm_persist_trace(eng.ctx.h, ctypes.c_void_p(buf.data_ptr()), cap), "trace")
eng.begin(x0, y0, {"maxiter": 12, "tolresid": 0.0, "maxtime": 1e9, "manviofun": manviofun,
                   "TRS_solver": "tCG", "second_order_stationarity": False})
eng.run_until(3)                       # warm
eng.advance(200)                      # one launch of 200 steps, traced
torch.cuda.synchronize()
hz = eng.lib.riptrm_device_clock_hz(eng.ctx.h)
t = buf.cpu().numpy().astype(np.float64) / hz * 1e6
for w in range(2):
    v = t[w]
    v = v[v[:, 0] > 0]
    tile = v[:, 1] - v[:, 0]
    bar = v[:, 2] - v[:, 1]
    state = v[:, 3] - v[:, 2]
    lean = v[v[:, 4] > 0]
    gather = lean[:, 4] - lean[:, 2]
    math = lean[:, 5] - lean[:, 4]
    stage = lean[:, 3] - lean[:, 5]
    raw = buf.cpu().numpy()[w]
    rl = raw[raw[:, 7] > 0]
    mhz = (rl[:, 7] - rl[:, 6]) / ((rl[:, 3] - rl[:, 0]) / hz) / 1e6 if len(rl) else np.array([0.0])
    step = np.diff(v[:, 0])
    print(json.dumps({"wg": "first" if w == 0 else "last", "steps": int(len(v)),
                      "tile_us": float(np.median(tile)), "barrier_us": float(np.median(bar)),
                      "state_us": float(np.median(state)),
                      "lean_steps": int(len(lean)), "gather_us": float(np.median(gather)) if len(lean) else None,
                      "math_us": float(np.median(math)) if len(lean) else None,
                      "stage_us": float(np.median(stage)) if len(lean) else None,
                      "core_clock_mhz": float(np.median(mhz)),
                      "tile_stamps_us": [float(np.median(v[v[:, q] > 0][:, q] - v[v[:, q] > 0][:, 0])) for q in (16, 17)
                                         if (v[:, q] > 0).any()],
                      "math_stamps_us": [float(np.median(lean[lean[:, 8 + q] > 0][:, 8 + q] - lean[lean[:, 8 + q] > 0][:, 4]))
                                         for q in range(7) if (lean[:, 8 + q] > 0).any()], "step_us": float(np.median(step)) if len(step) else None,
                      "p90_step_us": float(np.percentile(step, 90)) if len(step) else None}))
eng.ctx.check(eng.lib.riptrm_persist_trace(eng.ctx.h, None, 0), "trace off")
