"""Kernel stats (the rocprofv3 --stats summary) from a rocpd results database.

rocprofv3 on ROCm 7.2 writes `<dir>/<name>_results.db` (rocpd SQLite) by
default; this prints the same columns as its kernel_stats.csv:
usage: python3 rocpd_stats.py run_results.db > kernel_stats.csv
"""
import csv
import sqlite3
import statistics
import sys

db = sqlite3.connect(sys.argv[1])
rows = db.execute("select name, duration from kernels").fetchall()
by = {}
for name, dur in rows:
    by.setdefault(name, []).append(float(dur))
total = sum(sum(v) for v in by.values()) or 1.0
w = csv.writer(sys.stdout, quoting=csv.QUOTE_NONNUMERIC)
w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"])
for name, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
    w.writerow([name, len(v), int(sum(v)), sum(v) / len(v), 100.0 * sum(v) / total, int(min(v)), int(max(v)),
                statistics.pstdev(v)])
