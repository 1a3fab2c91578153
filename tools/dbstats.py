#!/usr/bin/env python3
"""Per-kernel duration stats (calls, average, min, max in ns) from a
rocprofv3 results database (`*_results.db`, the default output when no
--output-format is given). Usage: dbstats.py DB [--csv OUT]"""
import argparse
import csv
import sqlite3
import statistics

ap = argparse.ArgumentParser()
ap.add_argument("db")
ap.add_argument("--csv")
a = ap.parse_args()
c = sqlite3.connect(a.db)
by = {}
for name, dur in c.execute("select name, duration from kernels"):
    by.setdefault(name, []).append(dur)
rows = sorted(((n, len(v), sum(v), statistics.mean(v), min(v), max(v)) for n, v in by.items()),
              key=lambda r: -r[2])
for n, k, tot, avg, lo, hi in rows:
    print(f"{n[:60]:60s} {k:5d} {avg:11.0f} {lo:9d} {hi:9d}")
if a.csv:
    with open(a.csv, "w", newline="") as f:
        w = csv.writer(f, quoting=csv.QUOTE_ALL)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "MinNs", "MaxNs"])
        for r in rows:
            w.writerow([r[0], r[1], r[2], f"{r[3]:.1f}", r[4], r[5]])
