"""CPU side of the null-calibrated parity analysis (tests/parity.py null_*): for NonnegPCA instances
drawn by oracle/nonnegpca_gen.py, the oracle's reference run (dsymv) and its summation-order variants
(dgemv, dsymv on symmetric permutations P S P^T; parity.order_variants), each saved as JSON (log,
final x, y) under OUT/<seed>_<kind>.json.  A pool of single-threaded processes; runs already on disk
are skipped.  TEST INFRASTRUCTURE ONLY.

    python scripts/null_oracle_runs.py OUT N K SEED0 COUNT [WORKERS] [PERM_SEEDS...]
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]


def _plain(v):
    if v is None or isinstance(v, (str, bool, int)):
        return v
    if isinstance(v, np.bool_):
        return bool(v)
    if isinstance(v, np.integer):
        return int(v)
    return float(v)


def one(job):
    out, n, K, seed, kind = job
    path = os.path.join(out, f"{seed}_{kind}.json")
    if os.path.exists(path):
        return path
    from oracle import nonnegpca_gen as G
    from oracle import riptrm_oracle as O
    Z, x0, y0 = G.generate_instance(n, seed)
    S = Z + Z.T
    opt = dict(tolresid=0.0, maxtime=1e9, maxiter=K, manviofun=O.sphere_manvio)
    if kind == "ref":
        r = O.RIPTRMOracle(opt).run(O.NonnegPCAVectorized(S, S=S), x0, y0)
        x, y = r.x, r.y
    elif kind == "gemv":
        r = O.RIPTRMOracle(opt).run(O.NonnegPCAVectorized(S, S=S, symv=False), x0, y0)
        x, y = r.x, r.y
    else:
        p = np.random.RandomState(int(kind[1:])).permutation(n)
        Sp = np.ascontiguousarray(S[p][:, p])
        r = O.RIPTRMOracle(opt).run(O.NonnegPCAVectorized(Sp, S=Sp), x0[p], y0[p])
        inv = np.argsort(p)
        x, y = np.asarray(r.x)[inv], np.asarray(r.y)[inv]
    rec = {"seed": seed, "kind": kind, "log": {k: [_plain(v) for v in col] for k, col in r.log.items()},
           "tcg": [int(t["tcg_iters"]) for t in r.trace], "x": [float(v) for v in x], "y": [float(v) for v in y]}
    tmp = path + ".tmp"
    json.dump(rec, open(tmp, "w"))
    os.replace(tmp, path)
    return path


def main():
    out, n, K, seed0, count = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])
    workers = int(sys.argv[6]) if len(sys.argv) > 6 else 8
    perms = [int(v) for v in sys.argv[7:]] or [1, 2, 6, 7]
    os.makedirs(out, exist_ok=True)
    for v in ("OMP_NUM_THREADS", "OPENBLAS_NUM_THREADS", "MKL_NUM_THREADS"):
        os.environ[v] = "1"
    jobs = [(out, n, K, seed0 + b, kind) for b in range(count) for kind in ["ref", "gemv"] + [f"p{s}" for s in perms]]
    import concurrent.futures as cf
    import multiprocessing as mp
    with cf.ProcessPoolExecutor(max_workers=workers, mp_context=mp.get_context("spawn")) as ex:
        for i, p in enumerate(ex.map(one, jobs)):
            print(f"[{i + 1}/{len(jobs)}] {p}", flush=True)


if __name__ == "__main__":
    main()
