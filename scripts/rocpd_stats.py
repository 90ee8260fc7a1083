"""Kernel statistics (the rocprofv3 --stats CSV columns) from a rocprofv3 SQLite database (.db),
for runs made without --output-format csv.  Usage: python scripts/rocpd_stats.py <results.db> > stats.csv"""
import csv
import math
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
rows = {}
for name, dur in db.execute("select name, duration from kernels"):
    rows.setdefault(name, []).append(float(dur))
total = sum(sum(v) for v in rows.values())
w = csv.writer(sys.stdout, quoting=csv.QUOTE_NONNUMERIC)
w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"])
for name, v in sorted(rows.items(), key=lambda kv: -sum(kv[1])):
    m = sum(v) / len(v)
    sd = math.sqrt(sum((x - m) ** 2 for x in v) / len(v))
    w.writerow([name, len(v), sum(v), m, 100.0 * sum(v) / total, min(v), max(v), sd])
