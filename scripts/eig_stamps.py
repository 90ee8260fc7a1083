"""Per-phase device clocks of the hand-written eigensolver (csrc/riptrm_eig.h) on Exact_RepMat-like
matrices: RIPTRM_EIG_STAMPS=1 makes riptrm_sym_eig print them (matrix 0 of the batch) on stderr.

    RIPTRM_EIG_STAMPS=1 python scripts/eig_stamps.py M BATCH
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "riemannian-interior-point-trust-region-method_amd")]


def main():
    import torch
    import trs
    m, B = int(sys.argv[1]), int(sys.argv[2])
    rs = np.random.RandomState(m)
    mats = []
    for b in range(B):
        D = rs.randn(m, m) / np.sqrt(m)
        D = D + D.T
        if b % 2:
            D += np.diag(np.where(rs.rand(m) < 0.3, 10.0 ** rs.uniform(2, 6, m), 0.0))
        mats.append(D)
    A = torch.tensor(np.stack(mats), dtype=torch.float64, device="cuda")
    import ctypes
    ctx = trs._context(A.device)
    V = A.clone()
    w = torch.empty((B, m), dtype=torch.float64, device=A.device)
    info = torch.empty(B, dtype=torch.int32, device=A.device)
    p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    # vectors 1: eigenvectors of A; 2: of the tridiagonal form (the service's compact eigenvectors)
    for kind, mode in (("vectors", 1), ("compact", 2), ("values", 0)):
        for _ in range(3):
            V.copy_(A)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            ctx.check(ctx.lib.riptrm_sym_eig(ctx.h, m, B, p(V), m, m * m, p(w), m, p(info), mode), "riptrm_sym_eig")
            torch.cuda.synchronize()
            print(f"{kind}: m={m} batch={B} {1e3 * (time.perf_counter() - t0):.3f} ms", flush=True)


if __name__ == "__main__":
    main()
