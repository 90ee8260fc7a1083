"""Same-box A/B of Stiefel kernel builds (GPU): for each library (RIPTRM_LIB; tools/build_stiefel_variant.sh)
and environment setting, time projection and retraction of (n, p) x B points with HIP events and check
them against torch fp64 (projection: U - X sym(X^T U); retraction: Q^T Q = I and Q R = X + U with
R = Q^T (X + U) upper triangular with a positive diagonal).  One child process per variant (the library
is loaded once per process).  Prints one JSON line per (variant, B).

usage: python scripts/stiefel_ab.py n p B1,B2,... name=libpath[:ENV=VAL,...] ...
       (libpath "-" = the in-tree library)"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r"""
import json, os, sys, math
import torch
sys.path.insert(0, os.path.join(ROOT, "riemannian-interior-point-trust-region-method_amd"))
from stiefel import StiefelBatch
n, p = N_, P_
for B in BS_:
    g = torch.Generator(device="cuda"); g.manual_seed(1234 + B)
    X = torch.linalg.qr(torch.randn(B, n, p, dtype=torch.float64, device="cuda", generator=g))[0].contiguous()
    W = torch.randn(B, n, p, dtype=torch.float64, device="cuda", generator=g)
    st = StiefelBatch(n, p)
    ref = W - X @ (lambda m: (m + m.transpose(1, 2)) / 2)(X.transpose(1, 2) @ W)
    out = st.projection(X, W)
    perr = float((out - ref).abs().max() / ref.abs().max())
    U = (0.1 * ref).contiguous()
    Q = st.retraction(X, U)
    A = X + U
    R = Q.transpose(1, 2) @ A
    eye = torch.eye(p, dtype=torch.float64, device="cuda")
    orth = float((Q.transpose(1, 2) @ Q - eye).abs().max())
    low = float(torch.tril(R, -1).abs().max())
    diag_ok = bool((torch.diagonal(R, dim1=1, dim2=2) > 0).all())
    rec = float((Q @ torch.triu(R) - A).abs().max())
    res = {}
    for name, fn in (("proj", lambda: st.projection(X, W)), ("retr", lambda: st.retraction(X, U))):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        K = 20
        e0.record()
        for _ in range(K):
            fn()
        e1.record()
        torch.cuda.synchronize()
        res[name] = e0.elapsed_time(e1) * 1e3 / K
    floor = 3.0 * n * p * 8 * B / 8e12 * 1e6
    print(json.dumps({"variant": VAR_, "n": n, "p": p, "B": B, "proj_us": res["proj"], "retr_us": res["retr"],
                      "proj_frac": floor / res["proj"], "retr_frac": floor / res["retr"], "proj_err": perr,
                      "retr_orth": orth, "retr_lower": low, "retr_diag_pos": diag_ok, "retr_recon": rec}), flush=True)
"""


def main():
    n, p = int(sys.argv[1]), int(sys.argv[2])
    bs = [int(b) for b in sys.argv[3].split(",")]
    for spec in sys.argv[4:]:
        name, _, rest = spec.partition("=")
        lib, _, envs = rest.partition(":")
        env = dict(os.environ)
        if lib and lib != "-":
            env["RIPTRM_LIB"] = os.path.join(ROOT, lib)
        else:
            env.pop("RIPTRM_LIB", None)
        for kv in filter(None, envs.split(",")):
            k, _, v = kv.partition("=")
            env[k] = v
        code = (CHILD.replace("ROOT", repr(ROOT)).replace("N_", str(n)).replace("P_", str(p))
                .replace("BS_", repr(bs)).replace("VAR_", repr(name)))
        r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
        if r.returncode != 0:
            print(json.dumps({"variant": name, "error": r.stderr[-2000:]}), flush=True)
            continue
        sys.stdout.write(r.stdout)
        sys.stdout.flush()


if __name__ == "__main__":
    main()
