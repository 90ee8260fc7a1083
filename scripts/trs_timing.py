"""Latency of one device TRSgep (riptrm_trs_gep, 256 threads) vs dim and matrix kind (HIP events)."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "riemannian-interior-point-trust-region-method_amd"))
from trs import trs_gep_batched  # noqa: E402

for dim in (16, 40, 49, 96):
    for kind in ("pd", "indef"):
        rs = np.random.RandomState(dim)
        M = rs.randn(dim, dim)
        A = M @ M.T + np.eye(dim) if kind == "pd" else M + M.T
        for B in (1, 256):
            At = torch.tensor(np.broadcast_to(A, (B, dim, dim)).copy(), device="cuda")
            a = torch.tensor(rs.randn(B, dim), device="cuda")
            D = torch.full((B,), 100.0 if kind == "pd" else 0.5, dtype=torch.float64, device="cuda")
            trs_gep_batched(At, a, D)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                trs_gep_batched(At, a, D)
            e1.record()
            torch.cuda.synchronize()
            print(json.dumps({"dim": dim, "kind": kind, "batch": B, "us": e0.elapsed_time(e1) / 5 * 1e3}), flush=True)
