"""Offline null analysis: GPU logs (scripts/dump_gpu_logs.py) against the oracle runs of
scripts/null_oracle_runs.py, per instance: parity.check_null / null_summary, and the variants'
leave-one-out.  TEST INFRASTRUCTURE ONLY.

    python scripts/null_analyze.py GPU_DIR ORACLE_DIR [OUT_JSON]
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import parity as PY  # noqa: E402


class Run:
    def __init__(self, rec):
        self.log, self.x, self.y = rec["log"], np.array(rec["x"]), np.array(rec["y"])
        self.trace = [{"tcg_iters": t} for t in rec["tcg"]]


def main():
    gdir, odir = sys.argv[1], sys.argv[2]
    g = json.load(open(os.path.join(gdir, "logs.json")))
    xy = np.load(os.path.join(gdir, "xy.npz"))
    rows, names, vruns = [], [], []
    for b, inst in enumerate(g["instances"]):
        seed = inst["seed"]
        files = sorted(f for f in os.listdir(odir) if f.startswith(f"{seed}_") and f.endswith(".json"))
        if f"{seed}_ref.json" not in files or len(files) < 3:
            continue
        ra = Run(json.load(open(os.path.join(odir, f"{seed}_ref.json"))))
        vs = [Run(json.load(open(os.path.join(odir, f)))) for f in files if not f.endswith("_ref.json")]
        try:
            r = PY.check_null(inst["log"], ra, vs, xy["x"][b], xy["y"][b], inst["tcg"])
        except AssertionError as e:
            print("seed", seed, "row-by-row bar FAILED:", str(e)[:400])
            continue
        rows.append(r)
        names.append(f"seed {seed}")
        vruns.append(r["variants"])
    if not rows:
        return
    print(PY.null_summary(rows))
    for n, r in zip(names, rows):
        print(n, "gpu", r["gpu"]["div_row"], r["gpu"]["flip"], "/", r["gpu"]["rows"], "variants",
              [(v["div_row"], v["flip"] and v["flip"][1]) for v in r["variants"]],
              "dx %.1e/%.1e" % (r["gpu"]["dx"], max(v["dx"] for v in r["variants"])),
              "outer %.1e/%.1e" % (r["gpu"]["outer_dev"], max(v["outer_dev"] for v in r["variants"])),
              "cmp rows", r["rows_compared"], "exc", r["excursions"])
    print("LOO", PY.null_summary(PY.leave_one_out(vruns)))
    if len(sys.argv) > 3:
        PY.null_table(rows, names, PY.null_summary(rows), sys.argv[3])


if __name__ == "__main__":
    main()
