#!/usr/bin/env python3
"""Kernel statistics (the `rocprofv3 --stats` table) from a rocprofv3 rocpd SQLite db.

ROCm 7.2's rocprofv3 writes `<name>_results.db` by default; this prints the same
columns as its `kernel_stats.csv`, sorted by total duration.

    python tools/rocpd_stats.py gpurun_out/r01b/prof/run_results.db > profiles/r01/kernel_stats.csv
"""
import csv
import math
import sqlite3
import sys


def main(path):
    con = sqlite3.connect(path)
    rows = con.execute("select name, duration from kernels").fetchall()
    agg = {}
    for name, d in rows:
        agg.setdefault(name, []).append(int(d))
    total = sum(sum(v) for v in agg.values()) or 1
    w = csv.writer(sys.stdout, quoting=csv.QUOTE_NONNUMERIC)
    w.writerow(["Name", "Calls", "Duration (Nsec)", "Average (Nsec)", "Percent (Inc)", "Min (Nsec)",
                "Max (Nsec)", "Std_Dev"])
    for name, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        s = sum(v)
        mu = s / len(v)
        sd = math.sqrt(sum((x - mu) ** 2 for x in v) / len(v))
        w.writerow([name, len(v), s, mu, 100.0 * s / total, min(v), max(v), sd])


if __name__ == "__main__":
    main(sys.argv[1])
