"""Summarise the Stiefel PMC passes (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE over
tools/stiefel_stamps N P B) into profiles/r3_stiefel_pmc.json, the file bench.py's Stiefel leg reads
for `roofline.traffic`.  gfx950 correction (MI355X_MICROARCH.md, HBM/rocprofv3): the counters are
KiB per dispatch and FETCH_SIZE counts half the bytes of wide coalesced reads, so
read_bytes_corrected = 2 * FETCH_SIZE * 1024; write_bytes = WRITE_SIZE * 1024.

Usage: python scripts/stiefel_pmc_summary.py FETCH_CSV WRITE_CSV OUT --n 200 --p 50 --batch 256
"""
import argparse
import csv
import json
from collections import defaultdict


def per_kernel(path, counter):
    vals = defaultdict(list)
    with open(path) as fh:
        for r in csv.DictReader(fh):
            if r["Counter_Name"] != counter:
                continue
            name = r["Kernel_Name"].split("(")[0]
            if name.startswith("void "):
                name = name[5:]
            vals[name].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_csv")
    ap.add_argument("write_csv")
    ap.add_argument("out")
    ap.add_argument("--n", type=int, default=200)
    ap.add_argument("--p", type=int, default=50)
    ap.add_argument("--batch", type=int, default=256)
    a = ap.parse_args()
    f, w = per_kernel(a.fetch_csv, "FETCH_SIZE"), per_kernel(a.write_csv, "WRITE_SIZE")
    alg = {"read": 16 * a.n * a.p * a.batch, "write": 8 * a.n * a.p * a.batch}
    kernels = {}
    for k in sorted(set(f) & set(w)):
        if "riptrm_stiefel::" not in k:
            continue
        rb, wb = 2 * f[k] * 1024, w[k] * 1024
        kernels[k] = {"FETCH_SIZE": f[k], "WRITE_SIZE": w[k], "read_bytes_corrected": rb, "write_bytes": wb,
                      "traffic_over_algorithmic": (rb + wb) / (alg["read"] + alg["write"])}
    out = {"source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes) -- tools/stiefel_stamps {a.n} {a.p} "
                     f"{a.batch}; KiB per dispatch averaged over the dispatches of each kernel; FETCH_SIZE doubled "
                     "per MI355X_MICROARCH.md (gfx950 reports half of wide reads)",
           "n": a.n, "p": a.p, "B": a.batch,
           "algorithmic_bytes": {"proj": alg, "retr": alg},
           "kernels": kernels}
    json.dump(out, open(a.out, "w"), indent=1)
    for k, m in kernels.items():
        print(k, round(m["read_bytes_corrected"] / 1e6, 2), "MB read", round(m["write_bytes"] / 1e6, 2), "MB written",
              round(m["traffic_over_algorithmic"], 3), "x algorithmic")


if __name__ == "__main__":
    main()
