"""Summarise two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE) into profiles/ JSON.

Usage: python scripts/pmc_summarize.py FETCH_CSV WRITE_CSV OUT_SUMMARY OUT_TRAFFIC --n 4000 --batch 128

gfx950 correction (MI355X_MICROARCH.md, HBM/rocprofv3 section): FETCH_SIZE and WRITE_SIZE are KiB;
FETCH_SIZE counts half the bytes of wide coalesced streaming reads, so hbm_read = 2*FETCH_SIZE*1024.
The S-pass traffic figure is taken from the launch with the largest fetch (every instance active),
divided by its instance count (k_spass_sym: grid / (tiles x threads); k_spass_sup, a persistent grid:
--instances, the group size), and compared with the algorithmic bytes of one instance pass.
"""
import argparse
import csv
import json
from collections import defaultdict


def load(path, counter):
    rows = defaultdict(list)
    with open(path) as fh:
        for r in csv.DictReader(fh):
            if r["Counter_Name"] != counter:
                continue
            name = r["Kernel_Name"].split("(")[0]
            if name.startswith("void "):
                name = name[5:]
            name = name.split("<")[0]   # template instantiations count under their kernel's name
            if not name.startswith("riptrm::"):
                continue
            rows[name].append((int(r["Dispatch_Id"]), int(r["Grid_Size"]), float(r["Counter_Value"])))
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch")
    ap.add_argument("write")
    ap.add_argument("summary")
    ap.add_argument("traffic")
    ap.add_argument("--n", type=int, default=4000)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--threads", type=int, default=512, help="k_spass_sym workgroup size (instances = grid/(tiles*threads))")
    ap.add_argument("--instances", type=int, default=64,
                    help="instances in the max-traffic k_spass_sup launch (persistent grid: not derivable from it)")
    ap.add_argument("--source", default="")
    a = ap.parse_args()
    fetch, write = load(a.fetch, "FETCH_SIZE"), load(a.write, "WRITE_SIZE")
    ts = 128
    nt = (a.n + ts - 1) // ts
    wl = -(-(a.n - (nt - 1) * ts) // 32) * 32
    inst_stride = (nt - 1) * nt // 2 * ts * ts + (nt - 1) * ts * wl + wl * wl
    alg_pass = 8 * inst_stride + 16 * a.n           # S tiles once + x read + y write
    out = {"source": a.source,
           "correction": "FETCH_SIZE/WRITE_SIZE in KiB; hbm_read = 2*FETCH_SIZE*1024 (gfx950 wide-read undercount); "
                         "WRITE_SIZE as reported",
           "kernels": {}}
    for k in sorted(set(fetch) | set(write)):
        f = max(fetch.get(k, [(0, 0, 0.0)]), key=lambda t: t[2])
        w = max(write.get(k, [(0, 0, 0.0)]), key=lambda t: t[2])
        e = {"launches": len(fetch.get(k, [])), "grid": f[1],
             "max_launch_FETCH_SIZE_KiB": f[2], "max_launch_WRITE_SIZE_KiB": w[2],
             "hbm_read_bytes_corrected": 2 * f[2] * 1024, "hbm_write_bytes": w[2] * 1024}
        if k in ("riptrm::k_spass_sym", "riptrm::k_spass_sup"):
            inst = f[1] // (nt * (nt + 1) // 2 * a.threads) if k.endswith("sym") else a.instances
            e["instances_in_launch"] = inst
            e["algorithmic_bytes_per_launch"] = alg_pass * inst
            e["traffic_over_algorithmic"] = (e["hbm_read_bytes_corrected"] + e["hbm_write_bytes"]) / (alg_pass * inst)
        out["kernels"][k] = e
    with open(a.summary, "w") as fh:
        json.dump(out, fh, indent=1)
    kname = "k_spass_sup" if "riptrm::k_spass_sup" in out["kernels"] else "k_spass_sym"
    sp = out["kernels"].get("riptrm::" + kname)
    if sp:
        with open(a.traffic, "w") as fh:
            json.dump({"n": a.n, "layout": "sym", "kernel": kname,
                       "hbm_bytes_per_instance_pass": (sp["hbm_read_bytes_corrected"] + sp["hbm_write_bytes"])
                       / sp["instances_in_launch"],
                       "source": f"{a.summary} (max-traffic launch, {sp['instances_in_launch']} instances)"}, fh, indent=1)
    print(json.dumps(sp or {}))


if __name__ == "__main__":
    main()
