"""Stiefel kernel timing sweep (HIP events): projection / retraction / e2rh time vs batch and n."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "riemannian-interior-point-trust-region-method_amd"))
from stiefel import StiefelBatch  # noqa: E402


def timeit(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3  # us


out = []
for n, p in [(200, 50), (1000, 50), (200, 16), (4000, 64)]:
    for B in (256, 1024, 4096):
        if n * p * B * 8 * 3 > 8e9:
            continue
        st = StiefelBatch(n, p)
        X = torch.linalg.qr(torch.randn(B, n, p, dtype=torch.float64, device="cuda"))[0].contiguous()
        U = torch.randn(B, n, p, dtype=torch.float64, device="cuda")
        us_p = timeit(lambda: st.projection(X, U))
        us_r = timeit(lambda: st.retraction(X, 0.1 * U))
        gb = 3 * n * p * B * 8 / 1e9
        out.append({"n": n, "p": p, "batch": B, "proj_us": us_p, "proj_TBps": gb / (us_p * 1e-6) / 1e3,
                    "retr_us": us_r})
        print(json.dumps(out[-1]), flush=True)
