"""Section timing of k_state from an instrumented build (libriptrm_dbg.so, not shipped): device
wall-clock (100 MHz) offsets from kernel entry, averaged over instance 0's launches."""
import ctypes
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "riemannian-interior-point-trust-region-method_amd")
sys.path.insert(0, PKG)
import torch  # noqa: E402  (before the library: one HIP runtime in the process)
import riptrm_native as N  # noqa: E402

lib = N.load(os.path.join(PKG, "libriptrm_dbg.so"))
import engine  # noqa: E402
from problems import manviofun  # noqa: E402

n, B = int(sys.argv[1]), int(sys.argv[2])
eng = engine.NonnegPCABatch(n, B, log_capacity=64)
x, y = eng.generate_synthetic(20251212, ids=list(range(B)))
eng.begin(x, y, {"TRS_solver": "tCG", "second_order_stationarity": False, "maxiter": 12, "tolresid": 0.0,
                 "maxtime": math.inf, "manviofun": manviofun, "save_inner_iteration": False})
eng.run_until(12)
torch.cuda.synchronize()
out = (ctypes.c_double * 64)()
lib.riptrm_dbg_read.argtypes = [ctypes.c_void_p]
print("rc", lib.riptrm_dbg_read(ctypes.cast(out, ctypes.c_void_p)))
names = {0: "constructor", 2: "bsum x.u,x.d", 3: "bsum x.q", 4: "bsum d.Hd", 5: "bsum model", 6: "bsum r.r",
         7: "bsum x.dnew", 20: "before finish_write", 21: "end"}
for k in sorted(names):
    c = out[32 + k]
    print(f"{names[k]:>22}: {out[k] / max(c, 1) * 10:8.0f} ns after entry  ({int(c)} hits)")
