"""Summarise one rocprofv3 --pmc pass of the StableIdentification bench (k_si) into the issue
roofline bench.py's SI line reads (profiles/r5_si_pmc.json).

Usage: python scripts/si_pmc_summary.py COUNTER_CSV OUT_JSON --d 5 --source "..."

k_si is one wave per instance running a dependent chain of small d x d products (latency-bound: no
HBM or MFMA roof applies).  Its roof is the issue rate of one wave: at most one instruction per
cycle.  SQ_WAVE_CYCLES, SQ_ACTIVE_INST_ANY, SQ_WAIT_ANY and SQ_WAIT_INST_ANY count quad-cycles and
ACTIVE + WAIT + WAIT_INST ~= WAVE_CYCLES (MI355X_MICROARCH.md, PMC table): issue_frac =
ACTIVE_INST_ANY / WAVE_CYCLES is the fraction of a wave's lifetime in which it issues.  Sums over
every k_si dispatch of the pass (the bench's timed launch and its instrumented twin are identical
work).
"""
import argparse
import csv
import json
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("out")
    ap.add_argument("--d", type=int, default=5)
    ap.add_argument("--source", default="")
    a = ap.parse_args()
    tot = defaultdict(float)
    disp = set()
    for r in csv.DictReader(open(a.csv)):
        name = r["Kernel_Name"]
        if "k_si<" not in name and "k_si(" not in name:
            continue
        disp.add(int(r["Dispatch_Id"]))
        tot[r["Counter_Name"]] += float(r["Counter_Value"])
    wc = tot.get("SQ_WAVE_CYCLES", 0.0)
    out = {"source": a.source, "d": a.d, "kernel": "k_si", "dispatches": len(disp),
           "counters": dict(tot),
           "issue_frac": tot.get("SQ_ACTIVE_INST_ANY", 0.0) / wc if wc else None,
           "wait_frac": tot.get("SQ_WAIT_ANY", 0.0) / wc if wc else None,
           "wait_inst_frac": tot.get("SQ_WAIT_INST_ANY", 0.0) / wc if wc else None,
           "valu_insts_per_wave_cycle": (tot.get("SQ_INSTS_VALU", 0.0) / (4.0 * wc)) if wc else None,
           "definition": "issue_frac = SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES over every k_si dispatch (quad-cycle units "
                         "cancel); valu_insts_per_wave_cycle = SQ_INSTS_VALU / (4 x SQ_WAVE_CYCLES)"}
    json.dump(out, open(a.out, "w"), indent=1)
    print(json.dumps({k: out[k] for k in ("dispatches", "issue_frac", "wait_frac", "wait_inst_frac",
                                           "valu_insts_per_wave_cycle")}))


if __name__ == "__main__":
    main()
