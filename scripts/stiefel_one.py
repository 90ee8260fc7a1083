"""One Stiefel projection batch, a few times (short program for rocprofv3 --pmc passes)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "riemannian-interior-point-trust-region-method_amd"))
from stiefel import StiefelBatch  # noqa: E402

n, p, B = (int(v) for v in (sys.argv[1:4] if len(sys.argv) > 3 else (200, 50, 1024)))
st = StiefelBatch(n, p)
X = torch.randn(B, n, p, dtype=torch.float64, device="cuda") / n ** 0.5   # timing only (no hipSOLVER under --pmc)
U = torch.randn(B, n, p, dtype=torch.float64, device="cuda")
for _ in range(5):
    st.projection(X, U)
torch.cuda.synchronize()
print("ok")
