"""Summarise a rocprofv3 MFMA PMC pass (SQ_VALU_MFMA_BUSY_CYCLES, SQ_BUSY_CYCLES,
SQ_INSTS_VALU_MFMA_F64, GRBM_GUI_ACTIVE) into profiles/ JSON, per riptrm kernel.

Usage: python scripts/pmc_mfma_summarize.py PMC_CSV OUT_JSON [--source TEXT]

Per dispatch: counters are summed over their per-XCD / per-SE rows.  GRBM_GUI_ACTIVE is the sum
over the 8 XCDs (MI355X_MICROARCH.md, DVFS give-back), so the dispatch's wall in shader cycles is
GRBM_GUI_ACTIVE / 8 and its SIMD-cycles are that x 1024 SIMDs; mfma_busy_frac = MFMA busy cycles
/ SIMD-cycles.  cycles_per_mfma = busy / instructions (64 for v_mfma_f64_16x16x4_f64).
Dispatches are grouped by instruction count (full 128-column passes vs passes with compacted
second right-hand sides) so the figure of a full pass is not diluted by the solve's tail.
"""
import argparse
import csv
import json
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("out")
    ap.add_argument("--source", default="")
    a = ap.parse_args()
    per = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))
    with open(a.csv) as fh:
        for r in csv.DictReader(fh):
            name = r["Kernel_Name"].split("(")[0].replace("void ", "")
            if not name.startswith("riptrm::"):
                continue
            per[name][int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    out = {"source": a.source,
           "definition": "mfma_busy_frac = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE/8 * 1024 SIMDs); "
                         "counters summed per dispatch; groups by SQ_INSTS_VALU_MFMA_F64",
           "kernels": {}}
    for k, ds in sorted(per.items()):
        groups = defaultdict(list)
        for d in ds.values():
            groups[int(d.get("SQ_INSTS_VALU_MFMA_F64", 0))].append(d)
        e = {"dispatches": len(ds), "by_mfma_instructions": {}}
        for ins, lst in sorted(groups.items(), key=lambda t: -len(t[1]))[:6]:
            busy = sum(d.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) for d in lst) / len(lst)
            grbm = sum(d.get("GRBM_GUI_ACTIVE", 0) for d in lst) / len(lst)
            sqb = sum(d.get("SQ_BUSY_CYCLES", 0) for d in lst) / len(lst)
            e["by_mfma_instructions"][str(ins)] = {
                "dispatches": len(lst), "SQ_VALU_MFMA_BUSY_CYCLES": busy, "GRBM_GUI_ACTIVE": grbm,
                "SQ_BUSY_CYCLES": sqb,
                "cycles_per_mfma": busy / ins if ins else None,
                "mfma_busy_frac": busy / (grbm / 8 * 1024) if grbm else None}
        out["kernels"][k] = e
    with open(a.out, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out, indent=1)[:3000])


if __name__ == "__main__":
    main()
